"""Random-access roofline of the MI355X for the verdict engine's access shapes
(SURVEY.md §8(d) denominator 1).  Usage: python tools/gather_roofline.py"""
import ctypes as C
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libgather_probe.so")


def build():
    src = os.path.join(HERE, "gather_probe.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", src,
                               "-o", SO])


def main():
    build()
    L = C.CDLL(SO)
    L.probe_run.restype = C.c_float
    L.probe_run.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
    res = []
    n = 1 << 26
    for tb in (2 << 20, 32 << 20, 128 << 20, 4 << 30):
        for kind, name, bpa in ((0, "gather64", 64), (1, "gather4", 4), (2, "atomic8", 8)):
            for grid in (2048, 8192):
                ms = L.probe_run(kind, tb, n, grid, 3)
                res.append({"probe": name, "table_MiB": tb >> 20, "grid": grid, "ms": round(ms, 4),
                            "Gops": round(n / ms / 1e6, 2), "GBps_64B_lines": round(n * 64 / ms / 1e6, 1)})
                print(json.dumps(res[-1]), flush=True)
    ms = L.probe_run(3, 4 << 30, 0, 8192, 3)
    res.append({"probe": "stream16B", "table_MiB": 4096, "ms": round(ms, 4), "GBps": round((4 << 30) / ms / 1e6, 1)})
    print(json.dumps(res[-1]), flush=True)
    out = sys.argv[1] if len(sys.argv) > 1 else None
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
