"""Prices the parts of the config-5 IPv4 egress conntrack stage by timing-only
ablations (CV_ABLATE bits, cilium_amd/csrc/cv_dp.hpp); whole lxc_egress launches on a
2M-packet IPv4 batch after a warm-up that created the flows; interleaved rounds."""
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
    n = 1 << 21
    w = synth.config5(n, family=4)
    ctx, _ = H.product_ctx(w)
    f, l, _ = H.to_dev(w)
    src, fh = H.egress_inputs(w)
    out = {"ret": torch.empty(n, dtype=torch.int32, device="cuda:0"),
           "identity": torch.empty(n, dtype=torch.int32, device="cuda:0"),
           "ct": torch.empty(n, dtype=torch.uint8, device="cuda:0")}
    variants = {"full": 0, "no_delivery": 0x100, "no_policy": 0x200, "no_lookups": 0x300 | 0x400,
                "no_ctstore": 0x800, "one_per_group": 0x1000, "skeleton": 0x1f00, "no_pol_atomics": 0x1, "nat_defer_all": 0x2000}
    times = {k: [] for k in variants}
    for _ in range(2):
        ctx.lxc_egress(f, l, out, w.now, src_ep=src, flow_hash=fh)
    for rnd in range(4):
        for name, bits in variants.items():
            os.environ["CV_ABLATE"] = str(bits)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                ctx.lxc_egress(f, l, out, w.now, src_ep=src, flow_hash=fh)
            b.record()
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / 3)
    os.environ["CV_ABLATE"] = "0"
    res = {k: {"ms_median": round(float(np.median(v)), 3)} for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
