"""Agent-side cost of one map write becoming visible (cv_sync at the batch boundary)
on the config-2 tables: ipcache (102k prefixes) and the endpoint policy map (81k
entries).  Usage: python tools/sync_cost.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from cilium_amd import synth
    from tests import harness as H
    w = synth.config2(1 << 16)
    ctx, pm = H.product_ctx(w)
    res = {}
    for mode in ("incremental", "full"):
        if mode == "full":
            os.environ["CV_NO_INCREMENTAL"] = "1"
        for name in ("ipcache", "policy"):
            res[f"{name}_{mode}"] = measure(ctx, pm, w, name)
    print(json.dumps(res))


def measure(ctx, pm, w, name):
    import numpy as np
    if True:
        k, v = w.maps[name].keys, w.maps[name].vals
        idx = np.linspace(0, len(k) - 2, 1000).astype(int)    # every prefix length class
        ts = []
        for j in idx[::100]:
            t0 = time.perf_counter()
            assert pm[name].update(k[j].tobytes(), v[j].tobytes()) == 0
            ctx.sync()
            ts.append((time.perf_counter() - t0) * 1e3)
        res = {"entries": len(k), "ms_per_update_and_sync_median": round(float(np.median(ts)), 3)}
        t0 = time.perf_counter()
        for j in idx:
            assert pm[name].update(k[j].tobytes(), v[j].tobytes()) == 0
        ctx.sync()
        res["ms_1000_updates_one_sync"] = round((time.perf_counter() - t0) * 1e3, 2)
        return res


if __name__ == "__main__":
    main()
