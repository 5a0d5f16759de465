"""Trace notifications of the oracle (send_trace_notify, bpf/lib/trace.h:96-150),
checked on CPU against properties of the reference:

* every TRACE_TO_LXC pairs with the update_metrics(INGRESS, FORWARDED) beside it
  (trace.h:99-101), so their count equals the forwarded-ingress metric;
* every packet entering from-container gets one TRACE_FROM_LXC (bpf_lxc.c:681) and
  every packet passing the XDP prefilter one TRACE_FROM_* at from_netdev;
* MONITOR_AGGREGATION >= 1 hides exactly the FROM_* records, and >= 3 keeps a subset
  of those (the steps whose conntrack lookup asked for a report)."""
from __future__ import annotations

import numpy as np

from cilium_amd import synth
from tests import harness as H

KEY = ["packet", "subtype"]


def egress_run(w, agg, rounds=3):
    dp, _ = H.oracle_dp(w)
    dp.trace_attach(3 * w.n, agg)
    out = []
    for rnd in range(rounds):
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + 3 * rnd)
        tr, n = dp.trace_drain()
        assert len(tr) == n
        out.append((ref, np.sort(tr, order=KEY)))
    return dp, out


def as_set(tr):
    return {tuple(r) for r in tr.tolist()}


def test_config5_trace_streams():
    w = synth.config5(1 << 12, n_svc=100, n_ep=32, n_remote=64, seed=91)
    dp0, r0 = egress_run(w, 0)
    _, r1 = egress_run(w, 1)
    _, r3 = egress_run(w, 3)
    to_lxc = sum(int((tr["subtype"] == 0).sum()) for _, tr in r0)
    assert to_lxc == int(dp0.metrics()[0, 1, 0])                        # TRACE_TO_LXC <-> forwarded ingress
    valid = w.extra["src_ep"] < len(w.endpoints)
    for (ref, t0), (_, t1), (_, t3) in zip(r0, r1, r3):
        assert int((t0["subtype"] == 5).sum()) == int(valid.sum())      # one FROM_LXC per packet
        assert as_set(t1) == as_set(t0[t0["subtype"] < 5])              # level 1: FROM_* hidden
        assert as_set(t3) <= as_set(t1)                                 # level 3: a subset
        assert (t0["type"] == 4).all() and (t0["len_cap"] == np.minimum(t0["len_orig"], 128)).all()
    assert len(r3[1][1]) < len(r1[1][1]) < len(r1[0][1]) + len(r1[1][1])   # 3 s later: fewer reports
    assert len(r3[2][1]) > len(r3[1][1])                                    # 6 s later: interval elapsed


def test_config3_trace_streams():
    w = synth.config3(1 << 12, 1 << 10, n_ep=32, n_cidrs=512, n_ids=50, seed=13)
    dp, _ = H.oracle_dp(w)
    dp.trace_attach(3 * w.n, 0, 7)
    ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now)
    tr, n = dp.trace_drain()
    assert int((tr["subtype"] == 0).sum()) == int(dp.metrics()[0, 1, 0])
    frm = tr[tr["subtype"] >= 5]
    assert len(frm) == int((ref.xdp == 2).sum())                        # XDP_PASS -> from_netdev
    assert (frm["ifindex"] == 7).all() and (frm["source"] == 0).all()
