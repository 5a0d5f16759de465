"""Random 64-B line reads against table size and order (tools/gather_probe.hip): does a
multi-GiB conntrack table cost more per random line than the 4 GiB probe (address
translation reach), and what would sorting a batch's lookups by address give?
Measurement tool; usage: python tools/tlb_probe.py"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gather_roofline  # noqa: E402

gather_roofline.build()
L = C.CDLL(gather_roofline.SO)
L.probe_run.restype = C.c_float
L.probe_run.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
n = 1 << 24
for gib in (1, 4, 16, 32):
    for kind, name in ((0, "random"), (4, "sorted")):
        ms = L.probe_run(kind, gib << 30, n, 8192, 3)
        print(f"{gib:3d} GiB {name:7s} {n} lines {ms:8.3f} ms {n * 64 / (ms * 1e-3) / 1e9:8.1f} GB/s", flush=True)
