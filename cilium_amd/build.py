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
SOURCES = ["cv_ctx.cpp", "cv_kernels.hip", "cv_egress.hip", "cv_sort.hip", "cv_agent.cpp", "cv_epnode.cpp"]
ARCH = os.environ.get("CV_OFFLOAD_ARCH", "gfx950")


DEVICE_SOURCES = ["cv_kernels.hip", "cv_egress.hip", "cv_sort.hip", "cv_dev.hpp", "cv_dp.hpp", "cv_hash.hpp", "cv_lpm.hpp",
                  "cv_common.hpp"]


def kernel_sha():
    """Hash of the device-code sources (the .hip files and the headers they include):
    what a PMC traffic summary depends on; host-side changes leave it alone."""
    import hashlib
    h = hashlib.sha256()
    for f in DEVICE_SOURCES:
        with open(os.path.join(SRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(SRC, f) for f in os.listdir(SRC)] + [os.path.join(HERE, "..", "include", h) for h in ("cilium_hip.h", "cilium_agent.h", "cilium_epnode.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, out=OUT, defines=()):
    """Compile every source to an object in parallel, then link the shared library.
    Concurrent callers (one process per GPU) serialise on a lock file and re-check, so
    at most one of them compiles."""
    if not force and out == OUT and not needs_build():
        return out
    import fcntl
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and out == OUT and not needs_build():
            return out
        return _build(verbose, out, defines)


def _build(verbose, out, defines):
    base = ["/opt/rocm/bin/hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function"] + [f"-D{d}" for d in defines]
    objs, procs = [], []
    for src in SOURCES:
        obj = out + "." + os.path.splitext(src)[0] + ".o"
        cmd = base + ["-c", "-x", "hip", os.path.join(SRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    cmd = ["/opt/rocm/bin/hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    for o in objs:
        os.remove(o)
    os.replace(out + ".tmp", out)
    if out == OUT:
        try:
            build_c_caller(verbose)
        except (OSError, subprocess.CalledProcessError) as e:   # a test tool: never fails the product build
            print(f"[cilium_amd.build] tests/_bin/ct_walk not built: {e}", file=sys.stderr)
    return out


WALK_SRC = os.path.join(os.path.dirname(HERE), "tests", "ct_walk.c")
WALK_BIN = os.path.join(os.path.dirname(HERE), "tests", "_bin", "ct_walk")


def build_c_caller(verbose=False):
    """tests/_bin/ct_walk: a plain C caller of the C-ABI (the cgo glue's view), linked
    against the in-tree library (test tool, not product code)."""
    os.makedirs(os.path.dirname(WALK_BIN), exist_ok=True)
    cmd = ["gcc", "-O2", "-Wall", WALK_SRC, "-o", WALK_BIN, "-L" + os.path.dirname(OUT), "-lcilium_hip",
           "-Wl,-rpath," + os.path.dirname(OUT)]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
