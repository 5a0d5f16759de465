"""debug: config5 v4 (64-B records) egress, print CT4 rows that differ from the oracle"""
import sys, numpy as np
sys.path.insert(0, "/root/repo")
import torch
from cilium_amd import synth
from tests import harness as H
from tests.test_gpu_egress import run_egress

w = synth.config5(1 << 14, n_svc=1000, n_ep=128, n_remote=512, family=4, seed=51)
dev = "cuda:0"
dp, om = H.oracle_dp(w)
ctx, pm = H.product_ctx(w)
cuts = np.linspace(0, w.n, 3).astype(int)
for rnd in range(2):
    now = w.now + rnd * 3
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        o = run_egress(ctx, w, dev, lo, hi, now, False)
        ref = dp.lxc_egress(w.frames[lo:hi], w.length[lo:hi], w.extra["src_ep"][lo:hi], w.extra["flow_hash"][lo:hi], now=now)
        bad = sum(int((o[k] != getattr(ref, k)).sum()) for k in ("ret", "ct", "nl", "nu"))
        pk, pv = pm["ct4"].dump(); ok, ov = om["ct4"].dump()
        P = {bytes(k): bytes(v) for k, v in zip(pk, pv)}
        O = {bytes(k): bytes(v) for k, v in zip(ok, ov)}
        diff = [k for k in O if P.get(k) != O[k]]
        extra = [k for k in P if k not in O]
        print(f"round {rnd} batch {lo}-{hi}: verdict mismatches {bad}, ct rows {len(P)} vs {len(O)}, differing {len(diff)}, extra {len(extra)}")
        print(" gpu rows", len(pk), "unique", len(P), " oracle rows", len(ok), "unique", len(O))
        for k in diff[:2]:
            a, b = k[0:4], k[4:8]
            for kk, vv in list(zip(pk, pv)):
                kb = bytes(kk)
                if {kb[0:4], kb[4:8]} == {a, b}:
                    print("   gpu pair row", kb.hex(), bytes(vv).hex(), "ORA", O.get(kb, b"").hex())
            for kk in O:
                if {kk[0:4], kk[4:8]} == {a, b} and kk not in P:
                    print("   ora-only", kk.hex())
        for k in diff[:6]:
            pv_, ov_ = P.get(k), O[k]
            print(" key", k.hex(), "\n  gpu", pv_.hex() if pv_ else None, "\n  ora", ov_.hex())
        for k in extra[:3]:
            print(" extra", k.hex(), P[k].hex())
        if diff or extra:
            sys.exit(1)
