"""CT garbage collection on the GPU: cv_ct_gc over the config-3
conntrack table (16M flows -> ~32M entries incl. ICMP-RELATED twins), after one
ingress batch.  Times the C-ABI call (synchronous: launch + count readback) and the
kernel alone (HIP events), for a pure scan (time 0: nothing expires) and a GC that
deletes about half the entries.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cilium_amd import synth
    from tests import harness as H
    n_flows = int(os.environ.get("GC_FLOWS", 1 << 24))
    w = synth.config3(1 << 20, n_flows)
    ctx, pm = H.product_ctx(w)
    f, l, m = H.to_dev(w)
    out = H.dev_out(w.n, "cuda:0")
    ctx.netdev_ingress(f, l, out, w.now, mark=m)
    torch.cuda.synchronize()
    ct = pm["ct4"]
    life = np.ascontiguousarray(w.maps["ct4"].vals[:, 32:36]).view("<u4").ravel()
    res = {"flows": n_flows}
    for name, t in (("scan", 0), ("gc_half", int(np.median(life)) + 1)):
        t0 = time.perf_counter()
        deleted = ct.ct_gc(t)
        res[name] = {"time": t, "deleted": deleted, "ms_call": round((time.perf_counter() - t0) * 1e3, 3)}
    res["entries_after"] = len(ct)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
