"""Config 5 as one node across ranks with endpoint-owned CT maps (tests/ep_shard.py):
the prototype's merged result against one sequential run of the same per-endpoint-map
datapath -- every packet's verdict, drop reason, identity, CT result, proxy port and
lookup counts, every endpoint's CT4 and CT6 table, the policy counters, cilium_metrics.
CPU only (the oracle is every rank's datapath); the gloo variant exchanges the delivery
records between two processes."""
import os
import socket

import numpy as np
import pytest

from cilium_amd import synth
from tests import ep_shard as E
from tests import harness as H

CT_REPLY = 2


def _workload(n=1 << 12, seed=0xE5):
    # few endpoints: most flows stay on the node, services with local backends, replies
    return synth.config5(n, n_svc=120, n_ep=24, n_remote=32, seed=seed, vip_frac=0.5)


def _sequential(w):
    dp, maps = E.per_endpoint_dp(w)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    return ref, dp, maps


def _check(w, results, world):
    ref, dp, maps = _sequential(w)
    out, ct, metrics, (pk, pv) = E.merge(w, results)
    for k in E.RankState.FIELDS:
        bad = np.nonzero(out[k] != getattr(ref, k).astype(np.int64))[0]
        assert len(bad) == 0, (k, len(bad), bad[:5], out[k][bad[:5]], getattr(ref, k)[bad[:5]])
    for e in range(len(w.endpoints)):
        for fam, (keys, vals) in zip(("ct4", "ct6"), ct[e]):
            ok, ov = maps[fam][e].dump()
            a, b = H.sorted_rows(keys, vals), H.sorted_rows(ok, ov)
            assert a.shape == b.shape and (a == b).all(), (e, fam, H.rows_diff(a, b))
    assert (metrics == dp.metrics()).all()
    ok, ov = maps["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    # the dependency DESIGN.md §7 names: replies whose source program finds the entry
    # an earlier packet's delivery created on the replier's map, with the two endpoints
    # on different ranks
    src = w.extra["src_ep"].astype(int)
    deliv = ref.ret != -3
    cross_reply = (ref.ct == CT_REPLY) & deliv
    n_cross = 0
    for i in np.nonzero(cross_reply)[0]:
        dst = [d for d in E.candidates(w)[i]]
        n_cross += any(d % world != src[i] % world for d in dst)
    assert n_cross > 0
    assert sum(r["cross"] for r in results) > 0


@pytest.mark.parametrize("world", [2, 4])
def test_endpoint_owned_ct_simulated(world):
    w = _workload()
    results, rounds = E.simulate(w, world, w.now)
    print(f"world {world}: {w.n} packets in {rounds} exchange rounds")
    _check(w, results, world)
    assert rounds < w.n // 32                                      # rounds follow reply chains, not packets


def test_endpoint_owned_ct_at_capacity():
    """Maps sized so half of them fill within the batch (DROP_CT_CREATE_FAILED): the
    creates of different peers of one map compete for its room, so a map that may fill
    keeps packet order over all its operations (ep_shard.RankState._tight) -- ordering
    per (map, peer) alone differed from the sequential run in 48 of 4 096 packets."""
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=0xE5, vip_frac=0.5)
    w = synth.config5(1 << 12, ct_max=1 << 16, **kw)
    _, _, m0 = _sequential(w)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[len(sizes) // 2])
    w = synth.config5(1 << 12, ct_max=cap, **kw)
    results, rounds = E.simulate(w, 2, w.now)
    _check(w, results, 2)
    _, dp, maps = _sequential(w)
    full = sum(len(m) >= cap for fam in ("ct4", "ct6") for m in maps[fam])
    assert full >= 8 and dp.metrics()[155, 2, 0] + dp.metrics()[155, 1, 0] > 0, full


def test_candidates_cover_every_delivery():
    w = _workload(seed=0xE6)
    dp, _ = E.per_endpoint_dp(w)
    o, dl, _, _ = dp.lxc_egress_split(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    cand = E.candidates(w)
    deferred = np.nonzero(o.ret == E.DEFER)[0]
    assert len(deferred) > 0
    assert all(int(dl[i]) in cand[i] for i in deferred)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = _workload()
        st = E.RankState(w, rank, world, w.now)
        rounds = 0
        while True:
            box = st.progress()
            rounds += 1
            boxes = [None] * world
            dist.all_gather_object(boxes, box)                     # the exchange: delivery records
            for b in boxes:
                st.receive(b.get(rank, []))
            flags = [None] * world
            dist.all_gather_object(flags, st.done())
            if all(flags):
                break
        res = [None] * world
        dist.all_gather_object(res, st.result())
        if rank == 0:
            q.put((res, rounds))
    finally:
        dist.destroy_process_group()


def test_endpoint_owned_ct_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results, rounds = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    w = _workload()
    _check(w, results, 2)


# ---------------------------------------------------------------- the product scheduler (cv_epnode)
def host_node_ctx(w):
    """a host-only context (cv_open(-1)) holding w's service tables, endpoints with their
    own CT4 / CT6 maps and node config: what cv_epnode_open reads"""
    from cilium_amd import lib
    ctx = lib.Ctx(-1)
    for name in ("lb4_services", "lb6_services"):
        if name in w.maps:
            ctx.bind(name, ctx.map_from_spec(w.maps[name]))
    c4, c6 = w.maps["ct4"], w.maps["ct6"]
    handles = []
    for e in w.endpoints:
        m4 = ctx.map_create(c4.type, c4.key_size, c4.val_size, c4.max_entries)
        m6 = ctx.map_create(c6.type, c6.key_size, c6.val_size, c6.max_entries)
        i = ctx.endpoint_add(e["lxc_id"], e["seclabel"], None, m4)
        ctx.endpoint_config(i, ct6=m6, **H._ep_cfg(e))
        handles.append((m4.h, m6.h))
    if w.extra and "node" in w.extra:
        ctx.node_config(**w.extra["node"])
    return ctx, handles


def sched_simulate(w, world):
    """the endpoint-owned node with the product's round scheduler (cv_epnode_*, one per
    rank, lockstep rounds in-process) and the oracle as every rank's datapath; returns
    (results as RankState.result() gives them, rounds, stats of rank 0)"""
    from cilium_amd import lib
    now, src, fh = w.now, w.extra["src_ep"], w.extra["flow_hash"]
    ranks = []
    for r in range(world):
        ctx, handles = host_node_ctx(w)
        dp, maps = E.per_endpoint_dp(w)
        om = {}
        for e, (h4, h6) in enumerate(handles):
            om[h4], om[h6] = maps["ct4"][e], maps["ct6"][e]
        s = lib.EpSched(ctx, r, world, w.frames, src)
        s.set_counts(lambda hs, om=om: ([len(om[h]) for h in hs], [om[h].max_entries for h in hs]))
        ranks.append({"ctx": ctx, "dp": dp, "maps": maps, "s": s, "rec": {}, "mine": np.zeros(w.n, bool),
                      "out": {k: np.zeros(w.n, np.int64) for k in E.RankState.FIELDS}, "cross": 0})
    rounds = 0
    while sum(R["s"].pending() for R in ranks):
        rounds += 1
        assert rounds < w.n, "no progress"
        before = sum(R["s"].pending() for R in ranks)
        inbox = [[] for _ in range(world)]
        for r, R in enumerate(ranks):
            pk = R["s"].sources()
            dst = np.full(len(pk), -1, np.int32)
            recs = []
            if len(pk):
                o, dl, ifx, lab = R["dp"].lxc_egress_split(w.frames[pk], w.length[pk], src[pk], fh[pk], now=now)
                for j, i in enumerate(pk):
                    if o.ret[j] == E.DEFER:
                        dst[j] = int(dl[j])
                    else:
                        for k in E.RankState.FIELDS:
                            R["out"][k][i] = getattr(o, k)[j]
                        R["mine"][i] = True
                    recs.append({"frame": o.frames_out[j].copy(), "ifindex": int(ifx[j]), "label": int(lab[j]),
                                 "identity": int(o.identity[j]), "ct": int(o.ct[j]), "nl": int(o.nl[j]),
                                 "nu": int(o.nu[j])})
            rp, re_, rh, rpos, rr = R["s"].sources_done(pk, dst)
            at = 0
            for q, cnt in enumerate(rr):
                for j in range(at, at + int(cnt)):
                    inbox[q].append((int(rp[j]), int(re_[j]), int(rh[j]), recs[rpos[j]] if rh[j] else None, r))
                at += int(cnt)
        for q, R in enumerate(ranks):
            rows = inbox[q]
            if not rows:
                continue
            ops = R["s"].receive([x[0] for x in rows], [x[1] for x in rows], [x[2] for x in rows])
            for (i, d, has, rec, frm), op in zip(rows, ops):
                if op >= 0:
                    R["rec"][int(op)] = (i, d, rec)
                    R["cross"] += frm != q
        for R in ranks:
            ops, pk = R["s"].deliveries(2 * w.n + 16)
            if not len(ops):
                continue
            items = [R["rec"].pop(int(o)) for o in ops]
            assert [x[0] for x in items] == list(pk)
            o = R["dp"].lxc_deliver(np.stack([x[2]["frame"] for x in items]), w.length[pk], [x[1] for x in items],
                                    [x[2]["ifindex"] for x in items], [x[2]["label"] for x in items],
                                    [x[2]["nl"] for x in items], [x[2]["nu"] for x in items], now=now)
            for j, (i, _, rec) in enumerate(items):
                for k in ("ret", "proxy", "nl", "nu", "reason"):
                    R["out"][k][i] = getattr(o, k)[j]
                R["out"]["identity"][i] = rec["identity"]
                R["out"]["ct"][i] = rec["ct"]
                R["mine"][i] = True
        assert sum(R["s"].pending() for R in ranks) < before, f"round {rounds}: no operation could run"
    results = []
    for r, R in enumerate(ranks):
        owned = [e for e in range(len(w.endpoints)) if e % world == r]
        results.append({"out": {k: v[R["mine"]] for k, v in R["out"].items()}, "idx": np.nonzero(R["mine"])[0],
                        "ct": {e: (R["maps"]["ct4"][e].dump(), R["maps"]["ct6"][e].dump()) for e in owned},
                        "metrics": R["dp"].metrics(), "policy": R["maps"]["policy"].dump(), "cross": R["cross"]})
    st = ranks[0]["s"].stats()
    for R in ranks:
        R["s"].close()
        R["ctx"].close()
    return results, rounds, st


@pytest.mark.parametrize("world", [1, 2, 4])
def test_ep_sched_node(world):
    """the product's round scheduler (cv_epnode, C++) with the oracle as datapath: the
    ranks' merged result equals one sequential run"""
    w = _workload()
    results, rounds, st = sched_simulate(w, world)
    print(f"world {world}: {w.n} packets in {rounds} rounds, {st}")
    if world > 1:
        _check(w, results, world)
    else:
        ref, dp, maps = _sequential(w)
        out, ct, metrics, _ = E.merge(w, results)
        for k in E.RankState.FIELDS:
            assert (out[k] == getattr(ref, k).astype(np.int64)).all(), k
        assert (metrics == dp.metrics()).all()
    assert st["maps_ordered_whole_at_open"] == 0


def _sched_at_capacity(world, seed=0xE5, frac=0.5, n=1 << 12):
    """maps sized so that `frac` of them fill: the node run by the product's scheduler on
    `world` ranks against one sequential run -- every output, every map, metrics"""
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=seed, vip_frac=0.5)
    w = synth.config5(n, ct_max=1 << 16, **kw)
    _, _, m0 = _sequential(w)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[int(len(sizes) * (1 - frac))])
    w = synth.config5(n, ct_max=cap, **kw)
    results, rounds, st = sched_simulate(w, world)
    print(f"world {world} at capacity (seed {seed:#x}, {frac} full): {rounds} rounds, {st}")
    ref, dp, maps = _sequential(w)
    out, ct, metrics, _ = E.merge(w, results)
    for k in E.RankState.FIELDS:
        bad = np.nonzero(out[k] != getattr(ref, k).astype(np.int64))[0]
        assert len(bad) == 0, (k, len(bad), bad[:5])
    for e in range(len(w.endpoints)):
        for fam, (keys, vals) in zip(("ct4", "ct6"), ct[e]):
            ok, ov = maps[fam][e].dump()
            assert (H.sorted_rows(keys, vals) == H.sorted_rows(ok, ov)).all(), (e, fam)
    assert (metrics == dp.metrics()).all()
    return st, dp


@pytest.mark.parametrize("world", [1, 2])
def test_ep_sched_node_at_capacity(world):
    """maps sized so half of them fill: the scheduler orders a map that may fill over all
    its peers, and the node stays exact (48 of 4 096 packets differed without it)"""
    st, dp = _sched_at_capacity(world)
    assert st["maps_ordered_whole_at_open"] > 0 and dp.metrics()[155, 2, 0] + dp.metrics()[155, 1, 0] > 0


@pytest.mark.parametrize("seed,world,frac", [(0xE6, 3, 0.5), (0xE7, 2, 0.25), (0xE8, 4, 0.75), (0xE9, 3, 0.1)])
def test_ep_sched_node_at_capacity_sweep(seed, world, frac):
    """other seeds, odd and even rank counts (endpoint e on rank e % world) and other
    shares of full maps: exact every time"""
    _sched_at_capacity(world, seed, frac)


def test_ep_sched_node_index_follows_changes():
    """cv_epnode_open caches the node's address / service indexes per node view
    (cv::node_key: the context, its endpoint generation, the service maps bound and their
    versions, the loopback address).  A service whose backend moves to a local endpoint,
    and a new endpoint at an address packets already target, must show in the next
    batch's candidate destinations (the rows cv_epnode_sources_done lists per candidate)."""
    from cilium_amd import lib
    w = synth.config5(1 << 12, n_svc=200, n_ep=32, n_remote=128, seed=5, family=4)
    ctx = lib.Ctx(-1)
    lb = ctx.map_from_spec(w.maps["lb4_services"])
    ctx.bind("lb4_services", lb)
    c4, c6 = w.maps["ct4"], w.maps["ct6"]

    def add_ep(lxc_id, seclabel, cfg):
        m4 = ctx.map_create(c4.type, c4.key_size, c4.val_size, c4.max_entries)
        m6 = ctx.map_create(c6.type, c6.key_size, c6.val_size, c6.max_entries)
        i = ctx.endpoint_add(lxc_id, seclabel, None, m4)
        ctx.endpoint_config(i, ct6=m6, **cfg)
        return i

    for e in w.endpoints:
        add_ep(e["lxc_id"], e["seclabel"], H._ep_cfg(e))
    if w.extra and "node" in w.extra:
        ctx.node_config(**w.extra["node"])
    n, src = w.n, w.extra["src_ep"]
    dst = w.frames[:, 30:34].copy().view(">u4").reshape(-1)

    def cands():
        s = lib.EpSched(ctx, 0, 1, w.frames, src)
        rp, re_, _, _, _ = s.sources_done(np.arange(n, dtype=np.uint32), np.full(n, -1, np.int32))
        s.close()
        out = {}
        for p, e in zip(rp.tolist(), re_.tolist()):
            out.setdefault(p, set()).add(e)
        return out

    before = cands()
    assert before == cands()                                      # (the cached indexes: same answer)
    # a service's first backend moved to local endpoint 0 (10.0.1.0)
    keys = w.maps["lb4_services"].keys
    slave1 = np.nonzero((keys[:, 6] | keys[:, 7]) == 1)[0]
    vip_hit = [int(k) for k in slave1 if (dst == int.from_bytes(keys[k, 0:4].tobytes(), "big")).any()]
    k = keys[vip_hit[0]]
    vip = int.from_bytes(k[0:4].tobytes(), "big")
    rc, val = lb.lookup(k.tobytes())
    assert rc == 0
    val = bytearray(val)
    val[0:4] = (0x0A000100).to_bytes(4, "big")
    assert lb.update(k.tobytes(), bytes(val)) == 0
    after = cands()
    to_vip = np.nonzero(dst == vip)[0]
    assert len(to_vip) and all(0 in after.get(int(p), set()) for p in to_vip)
    # a new endpoint at a remote pod's address that packets target directly
    remote = np.nonzero((dst & 0xFFFF0000) == 0x0A100000)[0]
    addr = int(dst[remote[0]])
    ne = add_ep(9999, 0x2FFF, dict(ipv4=addr, ipv6=bytes(16), mac=H.DEFAULT_MAC, node_mac=H.NODE_MAC))
    again = cands()
    hit = np.nonzero(dst == addr)[0]
    assert all(ne in again.get(int(p), set()) for p in hit)
    assert all(ne not in after.get(int(p), set()) for p in hit)
    ctx.close()
