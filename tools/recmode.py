"""Times the config-2 kernel under the record-load modes (CV_RECMODE 0/1/2) with and
without the table work (CV_ABLATE), interleaved rounds in one process."""
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
    variants = {f"mode{mode}_{nm}": (mode, bits) for mode in (0, 1, 2) for nm, bits in (("full", 0), ("record_only", 15))}
    times = {k: [] for k in variants}
    for rnd in range(5):
        for name, (mode, bits) in variants.items():
            os.environ["CV_RECMODE"] = str(mode)
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
    res = {k: {"ms_median": round(float(np.median(v)), 4), "Gpps": round(n / np.median(v) / 1e6, 2)}
           for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
