"""Endpoints that do not share their maps: the launch parameters then carry no common
endpoint line (DpParams.uni4 / uni6) and every stage reads the packet's
own endpoint line.  Endpoints in G groups, each group with its own CT4 and CT6 maps
(per-endpoint conntrack, bpf_lxc.c's CT_MAP_TCP4 / CT_MAP_TCP6 when the endpoint's CT is
local: bpf/lib/conntrack_map.h) and every other group with its own copy of the policy
map (the per-endpoint POLICY_MAP, bpf/lib/maps.h); plus the shared-map workloads with the
common line switched off (CV_NO_UNI4).  Config 3 (netdev -> lxc ingress) and config 5
(from-container egress with local delivery): every output, every map of every group,
the metrics, against the oracle, bit-exact."""
import numpy as np
import pytest

from cilium_amd import synth
from tests import harness as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ING = ("xdp", "ret", "identity", "ct", "proxy", "nl", "nu", "reason")
EGR = ("ret", "reason", "identity", "ct", "proxy", "nl", "nu")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


def _grouped(w, groups, make_ctx):
    """(datapath, maps) with endpoint i on group i % groups: group 0 keeps the workload's
    CT maps (their preloaded flows), the other groups start empty; odd groups use their
    own copy of the policy map."""
    from oracle import oracle as O
    from cilium_amd import lib
    if make_ctx:
        dp = lib.Ctx(0, lib.F_DEFAULT)
        spec_map = dp.map_from_spec
        empty = dp.map_create
        add, cfg = dp.endpoint_add, dp.endpoint_config
    else:
        dp = O.ODp(O.F_DEFAULT)
        spec_map = O.OMap.from_spec
        empty = O.OMap
        add, cfg = dp.add_endpoint, dp.endpoint_config
    maps = {}
    for name, spec in w.maps.items():
        if name in ("ct4", "ct6"):
            continue
        maps[name] = spec_map(spec)
        if name in H.ROLE_NAMES:
            dp.bind(name, maps[name])
    per = {"ct4": [], "ct6": [], "policy": [maps["policy"]]}
    for g in range(groups):
        for name in ("ct4", "ct6"):
            s = w.maps.get(name)
            per[name].append(None if s is None else
                             spec_map(s) if g == 0 else empty(s.type, s.key_size, s.val_size, s.max_entries))
        if g % 2 == 1:
            per["policy"].append(spec_map(w.maps["policy"]))
    for i, e in enumerate(w.endpoints):
        g = i % groups
        pol = per["policy"][(g + 1) // 2 if g % 2 == 1 else 0]
        k = add(e["lxc_id"], e["seclabel"], pol, per["ct4"][g])
        cfg(k, ct6=per["ct6"][g], **H._ep_cfg(e))
    if w.extra and "node" in w.extra:
        dp.node_config(**w.extra["node"])
    if make_ctx:
        dp.sync()
    else:
        dp.keep += list(maps.values()) + [m for v in per.values() for m in v if m is not None]
    return dp, per


def _same_maps(pm, om):
    for name in ("ct4", "ct6", "policy"):
        for g, (a, b) in enumerate(zip(pm[name], om[name])):
            if a is None:
                continue
            ak, av = a.dump()
            bk, bv = b.dump()
            assert len(ak) == len(bk), (name, g, len(ak), len(bk))
            ra, rb = H.sorted_rows(ak, av), H.sorted_rows(bk, bv)
            assert (ra == rb).all(), (name, g, H.rows_diff(ra, rb))


def _check_fields(o, ref, fields, tag):
    for k in fields:
        bad = np.nonzero(o[k] != getattr(ref, k))[0]
        assert len(bad) == 0, (tag, k, bad[:5], o[k][bad[:5]], getattr(ref, k)[bad[:5]])


def _ingress_grouped(w, dev, groups, rounds):
    from tests.test_gpu_parity import run_ingress
    dp, om = _grouped(w, groups, False)
    ctx, pm = _grouped(w, groups, True)
    for r in range(rounds):
        wr = synth.Workload(w.name, w.maps, w.frames, w.length, w.mark, w.endpoints, now=w.now + r, extra=w.extra)
        o = run_ingress(ctx, wr, dev, 0, w.n, events=False)
        ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now + r)
        _check_fields(o, ref, ING, r)
        assert (ctx.metrics() == dp.metrics()).all(), r
    _same_maps(pm, om)
    assert sum(len(m) for m in pm["ct4"][1:]) > 0                  # the empty groups created flows
    ctx.close()


def _egress_grouped(w, dev, groups, rounds):
    from tests.test_gpu_egress import run_egress
    dp, om = _grouped(w, groups, False)
    ctx, pm = _grouped(w, groups, True)
    for r in range(rounds):
        o = run_egress(ctx, w, dev, 0, w.n, w.now + 3 * r, events=False)
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + 3 * r)
        _check_fields(o, ref, EGR, r)
        assert (ctx.metrics() == dp.metrics()).all(), r
    _same_maps(pm, om)
    assert sum(len(m) for m in pm["ct4"][1:]) > 0 and sum(len(m) for m in pm["ct6"][1:]) > 0
    ctx.close()


@pytest.mark.parametrize("groups", [2, 5])
def test_config3_endpoint_groups(dev, groups):
    w = synth.config3(1 << 16, 1 << 13, n_ep=128, n_cidrs=2048, n_ids=300, seed=71 + groups)
    _ingress_grouped(w, dev, groups, rounds=2)


def test_config3_endpoint_groups_dual_stack(dev):
    w = synth.config3(1 << 15, 1 << 12, n_ep=96, n_cidrs=2048, n_ids=300, seed=77, v6_frac=0.4)
    _ingress_grouped(w, dev, 3, rounds=2)


def test_config3_endpoint_groups_hot_runs(dev):
    """few address pairs: runs far over the in-register limit go through k_ct_hot with
    endpoints on different CT maps"""
    w = synth.config3(1 << 15, 64, n_ep=16, n_cidrs=512, n_ids=50, seed=78)
    _ingress_grouped(w, dev, 3, rounds=2)


@pytest.mark.parametrize("n", [1 << 15, 1 << 18])
def test_config3_merged_runs_across_maps(dev, monkeypatch, n):
    """Runs that hold members of different CT maps (advisor r04: two groups merged by a
    key collision): CV_COARSE_GROUPS keeps 8 bits of every group key, so each run of
    k_ct_hot mixes address pairs of endpoints on 5 CT maps; a member on another map than
    the run's first runs whole instead of folding into the run's map.  At 2^18 packets the
    runs pass HPAR_MIN members (the parallel elephant kernels cut them at their first
    member on another map or entry) and their bins pass LCAP (split keys ordered by
    k_gbin_tiles)."""
    monkeypatch.setenv("CV_COARSE_GROUPS", "1")
    w = synth.config3(n, 1 << 11, n_ep=40, n_cidrs=512, n_ids=60, seed=79)
    _ingress_grouped(w, dev, 5, rounds=2)


@pytest.mark.parametrize("groups", [2, 5])
def test_config5_endpoint_groups(dev, groups):
    w = synth.config5(1 << 15, n_svc=1000, n_ep=128, n_remote=512, seed=81 + groups)
    _egress_grouped(w, dev, groups, rounds=2)


def test_config5_endpoint_groups_hot_flows(dev):
    w = synth.config5(1 << 14, n_svc=40, n_ep=8, n_remote=16, n_flows=64, seed=88, odd_frac=5.0)
    _egress_grouped(w, dev, 3, rounds=3)


def test_shared_maps_without_common_line(dev, monkeypatch):
    """The workloads whose endpoints do share their maps, with the common line off: the
    per-packet endpoint reads the line replaced, on the same inputs."""
    from tests.test_gpu_egress import check_egress
    from tests.test_gpu_parity import check_ingress
    monkeypatch.setenv("CV_NO_UNI4", "1")
    check_ingress(synth.config3(1 << 15, 1 << 12, n_ep=128, n_cidrs=2048, n_ids=300, seed=91, v6_frac=0.3),
                  dev, batches=2, events=False)
    check_egress(synth.config5(1 << 14, n_svc=500, n_ep=64, n_remote=256, seed=92), dev, batches=2,
                 events=False)


def test_config3_per_endpoint_ct_admission(dev, capfd):
    """ConntrackLocal next to max_entries (verdict r04 item 3): 256 endpoints, each its
    own CT4 map (synth.per_endpoint_ct), connections concentrated on a few endpoints
    (ep_zipf) so dozens of maps start full while the others have room.  Each batch runs
    admitted at full width -- every map's walk one segment of the sorted scan -- with no
    one-packet launches; every output, every endpoint's map, metrics and policy counters
    against the oracle, over two batches (deletes after a policy change make room)."""
    import re
    w = synth.config3(1 << 18, 1 << 16, n_ep=256, n_cidrs=2048, n_ids=300, seed=83, ep_zipf=1.1)
    per = synth.per_endpoint_ct(w, 1 << 20)
    counts = np.array(sorted(len(s) for s in per))
    cap = int(counts[-40])                                       # the 40 busiest maps start full
    per = synth.per_endpoint_ct(w, cap)
    full0 = sum(len(s) >= cap for s in per)
    assert full0 >= 40
    dp, om = H.oracle_dp(w, ct_per_ep=per)
    ctx, pm = H.product_ctx(w, ct_per_ep=per)
    capfd.readouterr()
    import os
    os.environ["CV_ADMIT_STATS"] = "1"
    try:
        for r in range(2):
            if r == 1:                                           # the agent removes a third of the L4 rules
                pk, _ = om["policy"].dump()
                for k in pk[::3]:
                    if k[6]:
                        assert om["policy"].delete(k.tobytes()) == 0
                        assert pm["policy"].delete(k.tobytes()) == 0
            wr = synth.Workload(w.name, w.maps, w.frames, w.length, w.mark, w.endpoints, now=w.now + r, extra=w.extra)
            from tests.test_gpu_parity import run_ingress
            o = run_ingress(ctx, wr, dev, 0, w.n, events=False)
            ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now + r)
            _check_fields(o, ref, ING, r)
            assert (ctx.metrics() == dp.metrics()).all(), r
    finally:
        del os.environ["CV_ADMIT_STATS"]
    err = capfd.readouterr().err
    stats = re.findall(r"\[cv admit\] (\d+) packets in (\d+) windows, (\d+) passes", err)
    assert stats and all(int(p) == w.n for p, _, _ in stats), err[-2000:]    # whole-batch launches
    full = 0
    for a, b in zip(pm["ct4_ep"], om["ct4_ep"]):
        ak, av = a.dump()
        bk, bv = b.dump()
        assert len(ak) == len(bk)
        assert (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all()
        full += len(bk) == cap
    assert full >= 40
    ok, ov = om["policy"].dump()
    pk, pv = pm["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    m = dp.metrics()
    assert m[155, 1, 0] > 1000                                     # DROP_CT_CREATE_FAILED in the full maps
    ctx.close()


@pytest.mark.parametrize("events", [False, True])
def test_config5_per_endpoint_ct_admission(dev, monkeypatch, capfd, events):
    """ConntrackLocal on egress next to max_entries (verdict r04 item 3): every endpoint
    its own CT4 and CT6 map, sized so that about a third of them fill within the batch.
    A packet's source program creates in its source endpoint's map and its local delivery
    in the destination's: each launch runs admitted at full width (cv_ctx.cpp
    lxc_admitted_maps -- two budgets per packet, every map's walk a segment of the sorted
    scan, a pass that was not the sequential run undone from the copy-on-first-write slot
    set), with no one-packet launches.  Every output, every endpoint's two maps, metrics
    and policy counters against the oracle, over two batches (the second after the agent
    removed a third of the ingress L4 rules: denied established deliveries delete).  With
    events, the instance with the optional outputs: drop and trace records and the
    rewritten frames too (their rings' counts go back with an undone pass)."""
    import re
    from tests import ep_shard as E
    from tests.test_gpu_egress import run_egress
    from tests.test_gpu_ep_node import per_endpoint_ctx
    from tests.test_gpu_parity import same_frames, same_notifications, same_traces
    kw = dict(n_svc=4000, n_ep=192, n_remote=768, seed=87)
    n = 1 << 17
    w = synth.config5(n, ct_max=1 << 20, **kw)                   # the creates per map with room for all
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[len(sizes) * 2 // 3])
    w = synth.config5(n, ct_max=cap, **kw)
    dp, om = E.per_endpoint_dp(w)
    ctx, pm = per_endpoint_ctx(w)
    if events:
        ctx.notify_attach(w.n)
        dp.notify_attach(w.n)
        ctx.trace_attach(3 * w.n, 0)
        dp.trace_attach(3 * w.n, 0)
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    capfd.readouterr()
    for rnd in (0, 1):
        if rnd == 1:
            keys = w.maps["policy"].keys
            for k in keys[(keys[:, 6] != 0) & (keys[:, 7] == 0)][::3]:           # ingress, L4
                assert pm["policy"].delete(k.tobytes()) == 0 == om["policy"].delete(k.tobytes())
        now = w.now + 3 * rnd
        o = run_egress(ctx, w, dev, 0, w.n, now, events=events)
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=now, frames_out=events)
        _check_fields(o, ref, EGR, rnd)
        assert (ctx.metrics() == dp.metrics()).all(), rnd
        if events:
            assert same_notifications(ctx, dp) == int((o["reason"] != 0).sum())
            same_traces(ctx, dp, ref.ret)
            same_frames(o["frames_out"], ref.frames_out, w.frames)
    err = capfd.readouterr().err
    stats = re.findall(r"\[cv admit\] egress: (\d+) packets, (\d+) passes, (\d+) maps", err)
    assert stats and all(int(p) == w.n for p, _, _ in stats), err[-2000:]    # whole-batch launches
    full = 0
    for fam in ("ct4", "ct6"):
        for e, (a, b) in enumerate(zip(pm[fam], om[fam])):
            ak, av = a.dump()
            bk, bv = b.dump()
            assert len(ak) == len(bk), (fam, e, len(ak), len(bk))
            assert (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all(), (fam, e)
            full += len(bk) == cap
    assert full >= 40, full
    ok, ov = om["policy"].dump()
    pk, pv = pm["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    m = dp.metrics()
    assert m[155, 2, 0] + m[155, 1, 0] > 500                      # DROP_CT_CREATE_FAILED in the full maps
    ctx.close()


def test_per_endpoint_ct_room_bound(dev, monkeypatch, capfd):
    """ConntrackLocal with room (verdict r05 weak item 4: per-endpoint maps ran every launch
    through the admission passes, because no 64 000-entry map has room for 7 creates of
    EVERY packet of a launch).  The room check bounds each map's creates by the packets
    whose source or destination it is -- w_src per packet of its endpoint, w_dst per packet
    that may be delivered to it: the destination address's endpoint, or a backend of a
    service the packet may hit (CtBound, cv_dp.hpp) -- so these launches run at full width
    with no admission: config 5 (CT4 + CT6 per endpoint) and config 3 (CT4 per endpoint),
    every output, every map, metrics and policy counters against the oracle."""
    import re
    from tests import ep_shard as E
    from tests.test_gpu_egress import run_egress
    from tests.test_gpu_ep_node import per_endpoint_ctx
    from tests.test_gpu_parity import run_ingress
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    # config 5: 192 endpoints, 2^17 packets, maps of 2^16 entries (7 x 2^17 > 2^16: the global rule fails)
    w = synth.config5(1 << 17, n_svc=4000, n_ep=192, n_remote=768, seed=89, ct_max=1 << 16)
    dp, om = E.per_endpoint_dp(w)
    ctx, pm = per_endpoint_ctx(w)
    capfd.readouterr()
    for rnd in (0, 1):
        now = w.now + 3 * rnd
        o = run_egress(ctx, w, dev, 0, w.n, now, events=False)
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=now)
        _check_fields(o, ref, EGR, rnd)
        assert (ctx.metrics() == dp.metrics()).all(), rnd
    err = capfd.readouterr().err
    assert re.search(r"\[cv bound\] mode 1: \d+ packets, 384 maps, fits 1", err) and "[cv admit]" not in err, \
        err[-2000:]
    for fam in ("ct4", "ct6"):
        for e, (a, b) in enumerate(zip(pm[fam], om[fam])):
            ak, av = a.dump()
            bk, bv = b.dump()
            assert len(ak) == len(bk) and (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all(), (fam, e)
    ok, ov = om["policy"].dump()
    pk, pv = pm["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    ctx.close()
    # config 3: 256 endpoints each its own CT4 map of 2^16 entries, 2^17 packets (2 x 2^17 > 2^16)
    w = synth.config3(1 << 17, 1 << 14, n_ep=256, n_cidrs=2048, n_ids=300, seed=84)
    per = synth.per_endpoint_ct(w, 1 << 16)
    dp, om = H.oracle_dp(w, ct_per_ep=per)
    ctx, pm = H.product_ctx(w, ct_per_ep=per)
    capfd.readouterr()
    for rnd in (0, 1):
        wr = synth.Workload(w.name, w.maps, w.frames, w.length, w.mark, w.endpoints, now=w.now + rnd, extra=w.extra)
        o = run_ingress(ctx, wr, dev, 0, w.n, events=False)
        ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now + rnd)
        _check_fields(o, ref, ING, rnd)
        assert (ctx.metrics() == dp.metrics()).all(), rnd
    err = capfd.readouterr().err
    assert re.search(r"\[cv bound\] mode 0: \d+ packets, 256 maps, fits 1", err) and "[cv admit]" not in err, \
        err[-2000:]
    for a, b in zip(pm["ct4_ep"], om["ct4_ep"]):
        ak, av = a.dump()
        bk, bv = b.dump()
        assert len(ak) == len(bk) and (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all()
    ctx.close()


def test_config5_ep_zipf_per_endpoint_ct(dev, monkeypatch, capfd):
    """ConntrackLocal with a Zipf-popular client endpoint (`bench.py --workload config5
    --ct-local --ep-zipf 0.6` at 2^18 packets, verdict r05 item 4): the busiest endpoints'
    maps fill in the first step and stay full while the others keep room, as in the bench's
    steady state.  Three steps built the way bench.py builds them (synth.port_variant: a
    fifth of the flows take fresh client ports each step, so full maps see new creates fail
    next to closing connections freeing room); each launch over a full map runs admitted.
    Every output, every endpoint's CT4 / CT6 map, metrics and policy counters against the
    oracle after every step."""
    import copy
    import re
    from tests import ep_shard as E
    from tests.test_gpu_egress import run_egress
    from tests.test_gpu_ep_node import per_endpoint_ctx
    kw = dict(n_svc=8000, n_ep=512, n_remote=2048, seed=91, ep_zipf=0.6)
    n = 1 << 18
    w = synth.config5(n, ct_max=1 << 20, **kw)                   # the creates per map with room for all
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[-8])                                          # (the 8 busiest maps fill in step 1)
    w = synth.config5(n, ct_max=cap, **kw)
    dp, om = E.per_endpoint_dp(w)
    ctx, pm = per_endpoint_ctx(w)
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    capfd.readouterr()
    for v in (1, 2, 3):
        wv = copy.copy(w)
        wv.frames = H.apply_variant(w.frames, *synth.port_variant(w, v))
        now = w.now + v
        o = run_egress(ctx, wv, dev, 0, w.n, now, events=False)
        ref = dp.lxc_egress(wv.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=now)
        _check_fields(o, ref, EGR, v)
        assert (ctx.metrics() == dp.metrics()).all(), v
        full = 0
        for fam in ("ct4", "ct6"):
            for e, (a, b) in enumerate(zip(pm[fam], om[fam])):
                ak, av = a.dump()
                bk, bv = b.dump()
                assert len(ak) == len(bk), (v, fam, e, len(ak), len(bk))
                assert (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all(), (v, fam, e)
                full += len(bk) == cap
        assert full >= 4, (v, full)
    err = capfd.readouterr().err
    assert re.search(r"\[cv admit\] egress: \d+ packets, [2-9] passes", err), err[-2000:]   # (a pass undone)
    ok, ov = om["policy"].dump()
    pk, pv = pm["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    m = dp.metrics()
    assert m[155, 2, 0] + m[155, 1, 0] > 0                        # DROP_CT_CREATE_FAILED in the full maps
    ctx.close()
