"""Debug: output-frame differences (cv_out.frames_out vs the oracle) on small
config-3 and config-5 batches; prints the differing byte offsets of a few packets."""
import sys
import os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def show(name, got, ref, inp, extra=""):
    bad = np.nonzero((got != ref).any(axis=1))[0]
    print(name, "mismatching frames", len(bad), "of", len(got), extra)
    for i in bad[:4]:
        pos = np.nonzero(got[i] != ref[i])[0]
        print("  pkt", i, "pos", pos.tolist(), "got", got[i][pos].tolist(), "ref", ref[i][pos].tolist(),
              "in", inp[i][pos].tolist(), "changed(ref vs in)", np.nonzero(ref[i] != inp[i])[0].tolist())


def main():
    import torch
    from cilium_amd import synth
    from tests import harness as H
    w = synth.config3(1 << 12, 1 << 10, n_ep=32, n_cidrs=512, n_ids=50, seed=12)
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    f, l, m = H.to_dev(w, "cuda:0", 0, w.n)
    out = H.dev_out(w.n, "cuda:0")
    out["frames_out"] = torch.zeros(f.shape, dtype=torch.uint8, device="cuda:0")
    ctx.netdev_ingress(f, l, out, w.now, mark=m)
    o = H.host_out(out)
    ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now, frames_out=True)
    show("config3", o["frames_out"], ref.frames_out, w.frames, "ret eq %s" % (o["ret"] == ref.ret).all())
    w = synth.config5(1 << 12, n_svc=100, n_ep=32, n_remote=64, family=4, seed=51)
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    f, l, _ = H.to_dev(w, "cuda:0", 0, w.n)
    src, fh = H.egress_inputs(w, "cuda:0", 0, w.n)
    out = H.dev_out(w.n, "cuda:0")
    out["frames_out"] = torch.zeros(f.shape, dtype=torch.uint8, device="cuda:0")
    ctx.lxc_egress(f, l, out, w.now, src_ep=src, flow_hash=fh)
    o = H.host_out(out)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now, frames_out=True)
    show("config5", o["frames_out"], ref.frames_out, w.frames, "ret eq %s" % (o["ret"] == ref.ret).all())


if __name__ == "__main__":
    main()
