"""Runs the config-5 IPv4 egress path a few times on a 2M-packet batch (profiling driver)."""
import os
import sys

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
           "ct": torch.empty(n, dtype=torch.uint8, device="cuda:0")}
    for _ in range(4):
        ctx.lxc_egress(f, l, out, w.now, src_ep=src, flow_hash=fh)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
