"""FETCH_SIZE calibration for random 64-B line reads (MI355X_MICROARCH.md: "calibrate on
a known byte count in your own access pattern before trusting an absolute"): one
launch of tools/gather_probe.hip reading 2^26 random 64-B lines (4 GiB of lines) from
a 4 GiB table.  Run under `rocprofv3 --pmc FETCH_SIZE`; tools/pmc_summary.py divides
the known bytes by the counter.  Usage: python tools/pmc_calibrate.py"""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gather_roofline  # noqa: E402

gather_roofline.build()
L = C.CDLL(gather_roofline.SO)
L.probe_run.restype = C.c_float
L.probe_run.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
N = 1 << 26
ms = L.probe_run(0, 4 << 30, N, 8192, 1)
print(f"gather64 lines={N} bytes={N * 64} ms={ms:.3f}")
