"""Config 5 as ONE node across GPUs with endpoint-owned conntrack, on the HIP datapath
(cilium_amd/epnode.py): every endpoint its own CT4 and CT6 map (ConntrackLocal,
bpf_lxc.c:53-75), a packet's source program on its source's rank (cv_lxc_egress_split),
its local delivery on the destination's rank (cv_lxc_deliver) from the record exchanged
between them.  The ranks' merged result against one sequential run of the same
per-endpoint-map datapath on the oracle (tests/ep_shard.per_endpoint_dp): every packet's
verdict, drop reason, identity, CT result, proxy port and lookup counts, every endpoint's
CT4 and CT6 table, cilium_metrics and the policy counters.  One rank (every operation on
one GPU, in rounds) and two ranks as two processes on one GPU exchanging over gloo."""
import os
import socket

import numpy as np
import pytest

from cilium_amd import synth
from tests import ep_shard as E
from tests import harness as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


def _workload(n=1 << 12, seed=0xE5):
    # few endpoints: most flows stay on the node, services with local backends, replies
    return synth.config5(n, n_svc=120, n_ep=24, n_remote=32, seed=seed, vip_frac=0.5)


def per_endpoint_ctx(w, device=0):
    """the product context of w whose endpoints each own a fresh CT4 and CT6 map"""
    from cilium_amd import lib
    ctx = lib.Ctx(device, lib.F_DEFAULT)
    maps = {}
    for name, spec in w.maps.items():
        if name in ("ct4", "ct6"):
            continue
        maps[name] = ctx.map_from_spec(spec)
        if name in H.ROLE_NAMES:
            ctx.bind(name, maps[name])
    c4, c6 = w.maps["ct4"], w.maps["ct6"]
    maps["ct4"], maps["ct6"] = [], []
    for e in w.endpoints:
        m4 = ctx.map_create(c4.type, c4.key_size, c4.val_size, c4.max_entries)
        m6 = ctx.map_create(c6.type, c6.key_size, c6.val_size, c6.max_entries)
        i = ctx.endpoint_add(e["lxc_id"], e["seclabel"], maps["policy"], m4)
        ctx.endpoint_config(i, ct6=m6, **H._ep_cfg(e))
        maps["ct4"].append(m4)
        maps["ct6"].append(m6)
    if w.extra and "node" in w.extra:
        ctx.node_config(**w.extra["node"])
    ctx.sync()
    return ctx, maps


def _rank_run(w, rank, world, device, exchange=None, all_sum=None):
    from cilium_amd import epnode
    ctx, maps = per_endpoint_ctx(w, int(device.split(":")[1]))
    node = epnode.EpNode(ctx, rank, world, w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"],
                         device=device, exchange=exchange, all_sum=all_sum)
    rounds = node.run(w.now)
    out, idx = node.results()
    owned = [e for e in range(len(w.endpoints)) if e % world == rank]
    res = {"out": out, "idx": idx,
           "ct": {e: (maps["ct4"][e].dump(), maps["ct6"][e].dump()) for e in owned},
           "metrics": ctx.metrics(), "policy": maps["policy"].dump(), "cross": node.cross, "rounds": rounds,
           "launches": node.launches, "stats": node.sched.stats()}
    node.sched.close()
    ctx.close()
    return res


def _check(w, results):
    dp, maps = E.per_endpoint_dp(w)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    out = {k: np.zeros(w.n, np.int64) for k in E.RankState.FIELDS}
    seen = np.zeros(w.n, int)
    ct = {}
    metrics = np.zeros((256, 4, 2), np.uint64)
    for r in results:
        for k in E.RankState.FIELDS:
            out[k][r["idx"]] = r["out"][k]
        seen[r["idx"]] += 1
        ct.update(r["ct"])
        metrics += r["metrics"]
    assert (seen == 1).all(), "every packet finishes on exactly one rank"
    for k in E.RankState.FIELDS:
        want = getattr(ref, k).astype(np.int64)
        if k == "identity":
            want &= 0xFFFFFFFF
        bad = np.nonzero(out[k] != want)[0]
        assert len(bad) == 0, (k, len(bad), bad[:5], out[k][bad[:5]], want[bad[:5]])
    for e in range(len(w.endpoints)):
        for fam, (keys, vals) in zip(("ct4", "ct6"), ct[e]):
            ok, ov = maps[fam][e].dump()
            a, b = H.sorted_rows(keys, vals), H.sorted_rows(ok, ov)
            assert a.shape == b.shape and (a == b).all(), (e, fam, H.rows_diff(a, b))
    assert (metrics == dp.metrics()).all()
    # policy counters: every rank adds its deltas to the shared initial values
    init = H.sorted_rows(w.maps["policy"].keys, w.maps["policy"].vals)
    tot = init[:, 16:32].copy().view("<u8").reshape(-1, 2).copy()
    for r in results:
        rows = H.sorted_rows(*r["policy"])
        with np.errstate(over="ignore"):
            tot += rows[:, 16:32].copy().view("<u8").reshape(-1, 2) - init[:, 16:32].copy().view("<u8").reshape(-1, 2)
    got = init.copy()
    got[:, 16:32] = tot.view(np.uint8).reshape(-1, 16)
    ok, ov = maps["policy"].dump()
    assert (got == H.sorted_rows(ok, ov)).all()
    return ref


def test_endpoint_owned_one_rank(dev, capsys):
    """every operation on one GPU in rounds: the split source launches and the delivery
    launches reproduce one sequential run of the per-endpoint-map datapath"""
    w = _workload()
    res = _rank_run(w, 0, 1, dev)
    ref = _check(w, [res])
    assert (ref.ret == E.DEFER).sum() == 0 and res["rounds"] >= 2
    with capsys.disabled():
        print(f"\n  1 rank: {w.n} packets in {res['rounds']} rounds, {res['launches']} launches")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    from cilium_amd import epnode
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex, s = epnode.dist_exchange(world, rank, device=None)
        q.put((rank, _rank_run(_workload(), rank, world, "cuda:0", exchange=ex, all_sum=s)))
    finally:
        dist.destroy_process_group()


def test_endpoint_owned_two_ranks_gloo(dev, capsys):
    """two ranks (two processes on one GPU, records exchanged over gloo): the merged
    result equals one sequential run, with cross-rank deliveries among them"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    w = _workload()
    _check(w, [results[0], results[1]])
    assert sum(r["cross"] for r in results.values()) > 0
    with capsys.disabled():
        print(f"\n  2 ranks: {w.n} packets in {results[0]['rounds']} rounds, "
              f"{sum(r['cross'] for r in results.values())} cross-rank deliveries")


def test_split_then_deliver_at_capacity(dev, monkeypatch, capfd):
    """The two C-ABI halves next to max_entries on per-endpoint maps sized so half of them
    fill: every source program of a batch (cv_lxc_egress_split, one admitted launch per
    family), then every delivery record in packet order (cv_lxc_deliver, admitted: slot-1
    budgets, the same walks and slot log) -- against the oracle running the same two phases
    (or_lxc_egress_split, then or_lxc_deliver over the records in packet order): every
    output, every endpoint's CT4 / CT6 table, metrics.  (The endpoint-owned protocol's own
    ordering is exact while maps have room; next to a limit the creates of different peers
    of one map would have to keep packet order too)"""
    import re
    import torch
    from cilium_amd import epnode
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=0xE5, vip_frac=0.5)
    w = synth.config5(1 << 12, ct_max=1 << 16, **kw)
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[len(sizes) // 2])
    w = synth.config5(1 << 12, ct_max=cap, **kw)
    now = w.now
    # the oracle: both phases over the whole batch
    dp, om = E.per_endpoint_dp(w)
    o1, dl, ifx, lab = dp.lxc_egress_split(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=now)
    want = {k: getattr(o1, k).astype(np.int64).copy() for k in epnode.FIELDS}
    dsel = np.nonzero(o1.ret == epnode.DEFER)[0]
    o2 = dp.lxc_deliver(o1.frames_out[dsel], w.length[dsel], dl[dsel], ifx[dsel], lab[dsel], o1.nl[dsel], o1.nu[dsel],
                        now=now)
    for k in ("ret", "reason", "proxy", "nl", "nu"):
        want[k][dsel] = getattr(o2, k)
    # the HIP path: the same phases, per family (records of 64 / 128 B, as epnode.EpNode runs them)
    ctx, maps = per_endpoint_ctx(w, int(dev.split(":")[1]))
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    capfd.readouterr()
    node = epnode.EpNode(ctx, 0, 1, w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], device=dev)

    def host(o):
        r = {k: v.cpu().numpy().astype(np.int64) for k, v in o.items()}
        r["identity"] &= 0xFFFFFFFF
        r["proxy"] &= 0xFFFF
        return r
    got = {k: np.zeros(w.n, np.int64) for k in epnode.FIELDS}
    recs = {}
    for fam in (0, 1):
        sel = np.nonzero(node.v6 == (fam == 1))[0]
        f = node.fam[fam]
        out = node._dev_out(len(sel))
        buf = torch.zeros(len(sel) * epnode.REC, dtype=torch.uint8, device=dev)
        ctx.lxc_egress_split(f["frames"], f["length"], out, now, buf, src_ep=f["src_ep"], flow_hash=f["flow_hash"])
        o = host(out)
        r = buf.cpu().numpy().reshape(-1, epnode.REC)
        for k in epnode.FIELDS:
            got[k][sel] = o[k]
        recs[fam] = (sel[o["ret"] == epnode.DEFER], r[o["ret"] == epnode.DEFER])
    for fam in (0, 1):
        idx, rr = recs[fam]
        if not len(idx):
            continue
        out = node._dev_out(len(idx))
        rd = torch.from_numpy(np.ascontiguousarray(rr).reshape(-1)).to(dev)
        ctx.lxc_deliver(rd, len(idx), fam == 1, out, now)
        o = host(out)
        for k in ("ret", "reason", "proxy", "nl", "nu"):
            got[k][idx] = o[k]
    want["identity"] &= 0xFFFFFFFF
    for k in epnode.FIELDS:
        bad = np.nonzero(got[k] != want[k])[0]
        assert len(bad) == 0, (k, len(bad), bad[:5], got[k][bad[:5]], want[k][bad[:5]])
    for fam in ("ct4", "ct6"):
        for e, (a, b) in enumerate(zip(maps[fam], om[fam])):
            ak, av = a.dump()
            bk, bv = b.dump()
            assert (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all(), (fam, e, len(ak), len(bk))
    assert (ctx.metrics() == dp.metrics()).all()
    err = capfd.readouterr().err
    assert re.search(r"\[cv admit\] deliver: \d+ packets", err), err[-2000:]
    full = sum(len(m) >= cap for fam in ("ct4", "ct6") for m in om[fam])
    assert full >= 4 and dp.metrics()[155, 2, 0] + dp.metrics()[155, 1, 0] > 0, full
    ctx.close()


def test_endpoint_owned_at_capacity(dev, monkeypatch, capfd):
    """The endpoint-owned node next to max_entries (verdict r05 item 1): maps sized so half
    of them fill within the batch.  The scheduler orders a map that may fill over all its
    peers (include/cilium_epnode.h), the split source launches and the delivery launches
    run admitted, and every output, table, counter and metric equals the sequential
    per-endpoint-map oracle (59 of 4 096 verdicts differed with per-peer ordering alone)."""
    import re
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=0xE5, vip_frac=0.5)
    w = synth.config5(1 << 12, ct_max=1 << 16, **kw)
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[len(sizes) // 2])
    w = synth.config5(1 << 12, ct_max=cap, **kw)
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    capfd.readouterr()
    res = _rank_run(w, 0, 1, dev)
    _check(w, [res])
    err = capfd.readouterr().err
    assert re.search(r"\[cv admit\] deliver: \d+ packets", err), err[-2000:]
    dp, om = E.per_endpoint_dp(w)
    dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    full = sum(len(m) >= cap for fam in ("ct4", "ct6") for m in om[fam])
    assert full >= 8 and res["stats"]["maps_ordered_whole_at_open"] > 0, (full, res["stats"])
    m = dp.metrics()
    assert m[155, 2, 0] + m[155, 1, 0] > 0                        # DROP_CT_CREATE_FAILED
    with capfd.disabled():
        print(f"\n  at capacity: {w.n} packets, {res['rounds']} rounds, {full} maps full (max_entries {cap}), "
              f"{res['stats']}")


def _cap_main(rank, world, port, q):
    import torch.distributed as dist
    from cilium_amd import epnode
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex, s = epnode.dist_exchange(world, rank, device=None)
        q.put((rank, _rank_run(_cap_workload(), rank, world, "cuda:0", exchange=ex, all_sum=s)))
    finally:
        dist.destroy_process_group()


def _cap_workload():
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=0xE5, vip_frac=0.5)
    w = synth.config5(1 << 12, ct_max=1 << 16, **kw)
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    return synth.config5(1 << 12, ct_max=int(sizes[len(sizes) // 2]), **kw)


def test_endpoint_owned_at_capacity_two_ranks_gloo(dev, capsys):
    """the at-capacity node on two ranks (two processes on one GPU, gloo exchange)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cap_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    _check(_cap_workload(), [results[0], results[1]])
    with capsys.disabled():
        print(f"\n  2 ranks at capacity: {results[0]['rounds']} rounds, "
              f"{sum(r['cross'] for r in results.values())} cross-rank deliveries")


def test_deliver_on_fresh_context(dev):
    """cv_lxc_deliver on a context that never ran an egress launch (a rank whose endpoints
    only receive): its records' outputs equal the oracle's (advisor r05: the egress scratch
    the delivery launch writes was not allocated on such a context)."""
    import torch
    from cilium_amd import epnode
    w = _workload()
    dp, om = E.per_endpoint_dp(w)
    o1, dl, ifx, lab = dp.lxc_egress_split(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    # the records from a first context's split launch (IPv4 part)
    ctx1, _ = per_endpoint_ctx(w, int(dev.split(":")[1]))
    v6, rows = epnode.families(w.frames)
    idx = np.nonzero(~v6)[0]
    f = torch.from_numpy(np.ascontiguousarray(w.frames[idx, :64])).to(dev)
    ln = torch.from_numpy(w.length[idx].astype(np.uint32).view(np.int32)).to(dev)
    se = torch.from_numpy(w.extra["src_ep"][idx].astype(np.uint16).view(np.int16)).to(dev)
    fh = torch.from_numpy(w.extra["flow_hash"][idx].astype(np.uint32).view(np.int32)).to(dev)
    out = H.dev_out(len(idx), dev)
    buf = torch.zeros(len(idx) * epnode.REC, dtype=torch.uint8, device=dev)
    ctx1.lxc_egress_split(f, ln, out, w.now, buf, src_ep=se, flow_hash=fh)
    ret = out["ret"].cpu().numpy()
    sel = np.nonzero(ret == epnode.DEFER)[0]
    assert len(sel) > 0
    recs = buf.view(-1, epnode.REC)[torch.from_numpy(sel).to(dev)].contiguous()
    ctx1.close()
    # a fresh context runs only the deliveries
    ctx2, _ = per_endpoint_ctx(w, int(dev.split(":")[1]))
    o = H.dev_out(len(sel), dev)
    ctx2.lxc_deliver(recs.view(-1), len(sel), False, o, w.now)
    got = H.host_out(o)
    pk = idx[sel]
    dp, _ = E.per_endpoint_dp(w)                                    # (the deliveries' own fresh maps, as ctx2's)
    o2 = dp.lxc_deliver(o1.frames_out[pk], w.length[pk], dl[pk], ifx[pk], lab[pk], o1.nl[pk], o1.nu[pk], now=w.now)
    for k in ("ret", "reason", "proxy", "nl", "nu"):
        assert (got[k] == getattr(o2, k)).all(), k
    ctx2.close()
