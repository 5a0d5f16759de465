"""XCD-local vs device atomics for the policy counters (measurement tool)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gather_roofline as G  # noqa: E402


def main():
    G.build()
    L = C.CDLL(G.SO)
    L.probe_atomic_xcd.restype = C.c_float
    L.probe_atomic_xcd.argtypes = [C.c_uint64, C.c_uint64, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.probe_xcc_map.argtypes = [C.c_int, C.c_void_p]
    m = (C.c_uint32 * 64)()
    L.probe_xcc_map(64, m)
    print("xcc of blocks 0..63:", list(m))
    n = 1 << 25
    for nslots in (1 << 15, 1 << 18, 1 << 21):
        for scope, name in ((0, "workgroup"), (1, "agent")):
            ok = C.c_int(0)
            ms = L.probe_atomic_xcd(nslots, n, 8192, 3, scope, C.byref(ok))
            print(json.dumps({"slots_per_replica": nslots, "scope": name, "ms": round(ms, 4),
                              "Gatomics": round(n / ms / 1e6, 2), "sum_ok": bool(ok.value)}), flush=True)


if __name__ == "__main__":
    main()
