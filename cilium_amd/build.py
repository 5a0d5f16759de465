"""Builds the product library cilium_amd/_lib/libcilium_hip.so for gfx950 (in-tree).

hipcc cross-compiles without a GPU; the .so travels to the GPU box with the repo
snapshot.  Usage: python -m cilium_amd.build
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_lib", "libcilium_hip.so")
SOURCES = ["cv_ctx.cpp", "cv_kernels.hip", "cv_egress.hip"]
ARCH = os.environ.get("CV_OFFLOAD_ARCH", "gfx950")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(SRC, f) for f in os.listdir(SRC)] + [os.path.join(HERE, "..", "include", "cilium_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-x", "hip"] + [os.path.join(SRC, s) for s in SOURCES] + ["-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
