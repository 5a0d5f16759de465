"""Prices each part of a verdict kernel by timing-only ablations (CV_ABLATE bits,
cilium_amd/csrc/cv_dp.hpp) in one process, interleaved rounds (guide §5.4 rule 24)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cilium_amd import synth
    from tests import harness as H
    n = 1 << 24
    w = synth.config2(n)
    ctx, _ = H.product_ctx(w)
    f, l, m = H.to_dev(w)
    out = {"ret": torch.empty(n, dtype=torch.int32, device="cuda:0"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda:0")}
    variants = {"full": 0, "no_policy_atomics": 1, "no_ipcache": 2, "no_policy": 4, "no_metrics": 8,
                "no_atomics_no_metrics": 9, "no_ipcache_no_policy": 6, "record_only": 15}
    times = {k: [] for k in variants}
    for rnd in range(5):
        for name, bits in variants.items():
            os.environ["CV_ABLATE"] = str(bits)
            for _ in range(2):
                ctx.policy_ingress(0, f, l, out, mark=m)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                ctx.policy_ingress(0, f, l, out, mark=m)
            b.record()
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / 5)
    os.environ["CV_ABLATE"] = "0"
    res = {k: {"ms_median": round(float(np.median(v)), 4), "ms_min": round(float(np.min(v)), 4),
               "Gpps": round(n / np.median(v) / 1e6, 2)} for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
