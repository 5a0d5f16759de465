"""Config 4 by construction: conntrack sharded by address pair over ranks, tables
replicated, one collective (sum) for cilium_metrics; world_size 2 over gloo on
CPU.  Each rank runs its shard through a datapath (the CPU oracle here; the HIP
engine in the -m gpu variant) and rank 0 checks the merged result -- verdicts,
CT tables, policy counters, metrics -- against one unsharded sequential run."""
import os
import socket

import numpy as np
import pytest

from cilium_amd import shard, synth
from tests import harness as H


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload():
    return synth.config3(1 << 13, 1 << 11, n_ep=64, n_cidrs=1024, n_ids=100, seed=41)


def _rank_main(rank, world, port, use_gpu, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = _workload()
        part, own = shard.split_workload(w, world, rank)
        if use_gpu:
            ctx, maps = H.product_ctx(part, device=0)
            f, l, m = H.to_dev(part, "cuda:0")
            out = H.dev_out(part.n, "cuda:0")
            ctx.netdev_ingress(f, l, out, part.now, mark=m)
            o = H.host_out(out)
            res = {k: o[k] for k in ("ret", "identity", "ct", "reason")}
            met = ctx.metrics()
        else:
            dp, maps = H.oracle_dp(part)
            ref = dp.netdev_ingress(part.frames, part.length, part.mark, now=part.now)
            res = {k: getattr(ref, k) for k in ("ret", "identity", "ct", "reason")}
            met = dp.metrics()
        t = torch.from_numpy(met.astype(np.int64).reshape(-1))
        shard.allreduce_counters(t)                      # the one cross-rank collective
        ck, cv = maps["ct4"].dump()
        pk, pv = maps["policy"].dump()
        mine = {"own": own, "res": res, "ct": (ck, cv), "pol": (pk, pv)}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        if rank == 0:
            q.put({"metrics": t.numpy().reshape(256, 4, 2), "parts": gathered})
        if use_gpu:
            ctx.close()
    finally:
        dist.destroy_process_group()


def _run(world, use_gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, use_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


def _check(out):
    w = _workload()
    dp, om = H.oracle_dp(w)
    ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now)
    got = {k: np.zeros_like(getattr(ref, k)) for k in ("ret", "identity", "ct", "reason")}
    seen = np.zeros(w.n, bool)
    for part in out["parts"]:
        for k in got:
            got[k][part["own"]] = part["res"][k]
        seen[part["own"]] = True
    assert seen.all()
    for k in got:
        assert (got[k] == getattr(ref, k)).all(), k
    assert (out["metrics"] == dp.metrics().astype(np.int64)).all()
    ck = np.concatenate([p["ct"][0] for p in out["parts"]])
    cv = np.concatenate([p["ct"][1] for p in out["parts"]])
    ok, ov = om["ct4"].dump()
    assert len(ck) == len(ok)
    assert (H.sorted_rows(ck, cv) == H.sorted_rows(ok, ov)).all()
    # policy counters: the agent sums them over ranks
    ok, ov = om["policy"].dump()
    tot = np.zeros((len(ok), 2), np.uint64)
    for p in out["parts"]:
        pk, pv = p["pol"]
        rows = H.sorted_rows(pk, pv)
        assert (rows[:, :8] == H.sorted_rows(ok, ov)[:, :8]).all()
        tot += rows[:, 16:32].copy().view("<u8").reshape(-1, 2)
    want = H.sorted_rows(ok, ov)[:, 16:32].copy().view("<u8").reshape(-1, 2)
    assert (tot == want).all()


def test_shard_key_is_direction_symmetric():
    w = _workload()
    f = w.frames.copy()
    f[:, 26:30], f[:, 30:34] = w.frames[:, 30:34], w.frames[:, 26:30]
    for world in (2, 3, 8):
        assert (shard.flow_shard(w.frames, w.length, world) == shard.flow_shard(f, w.length, world)).all()
    keys = w.maps["ct4"].keys
    rk = keys.copy()
    rk[:, 0:4], rk[:, 4:8] = keys[:, 4:8], keys[:, 0:4]
    assert (shard.ct4_shard(keys, 8) == shard.ct4_shard(rk, 8)).all()


def test_two_ranks_gloo_oracle():
    _check(_run(2, use_gpu=False))


@pytest.mark.gpu
def test_two_ranks_gloo_hip():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check(_run(2, use_gpu=True))


def test_sharded_oracle_threads_equal_sequential():
    """bench.py's CPU baseline for the conntrack paths: the oracle partitioned by
    address pair over host threads (tests/harness.ShardedOracle) gives the sequential
    run's verdicts, CT4 / CT6 tables and counters, IPv6 pairs included, over two
    batches (the second one with fresh client ports, synth.port_variant)."""
    w = synth.config3(1 << 13, 1 << 10, n_ep=64, n_cidrs=1024, n_ids=100, seed=43, v6_frac=0.3)
    dp, om = H.oracle_dp(w)
    so = H.ShardedOracle(w, 4)
    for v in (0, 1):
        f = H.apply_variant(w.frames, *synth.port_variant(w, v))
        ref = dp.netdev_ingress(f, w.length, w.mark, now=w.now + v)
        got, _ = so.netdev_ingress(f, now=w.now + v)
        for k in ("ret", "identity", "ct", "reason", "nl", "nu", "proxy"):
            assert (getattr(got, k) == getattr(ref, k)).all(), (v, k)
    assert (so.metrics() == dp.metrics()).all()
    for name in ("ct4", "ct6"):
        ck, cv = so.dump(name)
        ok, ov = om[name].dump()
        assert len(ck) == len(ok) and (H.sorted_rows(ck, cv) == H.sorted_rows(ok, ov)).all(), name


def test_config4_ranks_hold_disjoint_parts_of_one_flow_set():
    """bench.py's config 3 / 4 at N > 1: every rank draws the same candidate flows and
    keeps the address pairs it owns, so the CT shards are disjoint, every packet is
    its rank's, and the union is one flow set (a rank's flows are found in no other
    rank's shard, reply and RELATED entries included)."""
    world, n = 3, 1 << 14
    parts = [synth.config3(n, n, n_ep=64, n_cidrs=1024, n_ids=100, seed=7, shard=(r, world)) for r in range(world)]
    seen, total = set(), 0
    for r, w in enumerate(parts):
        assert (shard.flow_shard(w.frames, w.length, world) == r).all()
        keys = w.maps["ct4"].keys
        assert (shard.ct4_shard(keys, world) == r).all()
        mine = set(map(bytes, keys))                     # (a pair's RELATED twin repeats: one entry)
        assert not (mine & seen)
        seen |= mine
        total += len(mine)
    assert len(seen) == total


def test_table_digest_matches_oracle():
    """tests/harness.table_digest (numpy, over a device dump) is the oracle's
    or_map_digest: the full-size GPU tests compare 33M-entry tables through it."""
    w = synth.config3(1 << 12, 1 << 12, n_ep=64, n_cidrs=1024, n_ids=100, seed=3)
    dp, om = H.oracle_dp(w)
    dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now)
    for name in ("ct4", "policy"):
        k, v = om[name].dump()
        assert om[name].digest() == H.table_digest(k, v)
        assert om[name].digest()[0] == len(k) > 0
    k, v = om["ct4"].dump()
    v2 = v.copy()
    v2[0, 0] ^= 1
    assert H.table_digest(k, v2) != H.table_digest(k, v)


# ---------------------------------------------------------------- config 5: replicas
# bench.py --workload config5 at N > 1 runs N independent nodes (an
# exact conntrack sharding of the egress path needs cross-rank ordering): every rank
# holds the replicated tables and its own conntrack, verdicts its own batch (here rank
# r: the batch with fresh client ports, synth.port_variant(w, r + 1)), and the one
# collective sums cilium_metrics.

def _c5_workload():
    return synth.config5(1 << 12, n_svc=400, n_ep=64)


def _c5_batch(w, rank):
    return H.apply_variant(w.frames, *synth.port_variant(w, rank + 1))


def _c5_rank_main(rank, world, port, use_gpu, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = _c5_workload()
        frames = _c5_batch(w, rank)
        wr = synth.Workload(w.name, w.maps, frames, w.length, w.mark, w.endpoints, now=w.now, extra=w.extra)
        if use_gpu:
            from tests.test_gpu_egress import run_egress
            ctx, maps = H.product_ctx(wr, device=0)
            o = run_egress(ctx, wr, "cuda:0", 0, wr.n, wr.now, events=False)
            res = {k: o[k] for k in ("ret", "identity", "ct", "reason")}
            met = ctx.metrics()
        else:
            dp, maps = H.oracle_dp(wr)
            ref = dp.lxc_egress(frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
            res = {k: getattr(ref, k) for k in ("ret", "identity", "ct", "reason")}
            met = dp.metrics()
        mine = torch.from_numpy(met.astype(np.int64).reshape(-1))
        t = mine.clone()
        shard.allreduce_counters(t)                      # the one cross-rank collective
        ct = [maps[n].dump() for n in ("ct4", "ct6")]
        gathered = [None] * world
        dist.all_gather_object(gathered, {"res": res, "ct": ct, "met": mine.numpy()})
        if rank == 0:
            q.put({"metrics": t.numpy().reshape(256, 4, 2), "ranks": gathered})
        if use_gpu:
            ctx.close()
    finally:
        dist.destroy_process_group()


def _c5_check(out, world):
    w = _c5_workload()
    total = np.zeros((256, 4, 2), np.int64)
    for rank, got in enumerate(out["ranks"]):
        dp, om = H.oracle_dp(w)                          # the rank's own node: fresh tables and conntrack
        ref = dp.lxc_egress(_c5_batch(w, rank), w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
        for k in ("ret", "identity", "ct", "reason"):
            assert (got["res"][k] == getattr(ref, k)).all(), (rank, k)
        for name, (ck, cv) in zip(("ct4", "ct6"), got["ct"]):
            ok, ov = om[name].dump()
            assert len(ck) == len(ok) and (H.sorted_rows(ck, cv) == H.sorted_rows(ok, ov)).all(), (rank, name)
        assert (got["met"].reshape(256, 4, 2) == dp.metrics().astype(np.int64)).all()
        total += dp.metrics().astype(np.int64)
    assert (out["metrics"] == total).all()               # the all_reduce = the nodes' sum


def _c5_run(world, use_gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_rank_main, args=(r, world, port, use_gpu, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


def test_config5_replicas_gloo_oracle():
    _c5_check(_c5_run(2, use_gpu=False), 2)


@pytest.mark.gpu
def test_config5_replicas_gloo_hip():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _c5_check(_c5_run(2, use_gpu=True), 2)


@pytest.mark.gpu
def test_bench_two_ranks_gloo(tmp_path):
    """bench.py's N > 1 path, executed before any 8-GPU node runs it: two spawned ranks
    (WORLD_SIZE=2, both on GPU 0, gloo instead of RCCL) through the init, the per-rank
    shard draw, the barriers, the MAX-reduce of the elapsed time and the cilium_metrics
    all_reduce.  One JSON line (rank 0) with n_gpus 2; the ranks' packets lie on
    disjoint address pairs (config 4: conntrack sharded by pair); the reduced metrics
    equal the sum of the two ranks' own."""
    import json
    import subprocess
    import sys
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "config3",
             "--packets", "65536", "--flows", "65536", "--steps", "2", "--warmup", "1", "--no-cpu",
             "--dist-backend", "gloo", "--dump", str(tmp_path)],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [l for l in outs[0][0].splitlines() if l.strip()]
    assert len(lines) == 1 and not outs[1][0].strip()
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["ct_slot_load"]["ct4"][0] > 0
    d = [np.load(tmp_path / f"rank{r}.npz") for r in range(2)]
    assert len(np.intersect1d(d[0]["pair_keys"], d[1]["pair_keys"])) == 0
    for r in range(2):                                              # every packet on a pair its rank owns
        assert (d[r]["pair_keys"] % np.uint64(2) == r).all()
    total = d[0]["metrics_local"] + d[1]["metrics_local"]
    assert total.sum() > 0
    assert (d[0]["metrics_reduced"] == total).all() and (d[1]["metrics_reduced"] == total).all()
    assert d[0]["elapsed"] == d[1]["elapsed"]                       # the MAX over ranks


@pytest.mark.gpu
def test_bench_ep_owned_two_ranks_gloo():
    """bench.py --ep-owned at N = 2 (config 5 as one node: two spawned ranks on GPU 0, gloo
    instead of RCCL): the rounds, the per-round exchange and the reductions run, one JSON
    line (rank 0) with the node's packets, rounds and cross-rank deliveries."""
    import json
    import subprocess
    import sys
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "config5", "--ep-owned",
             "--packets", "16384", "--ct-local", "2048", "--steps", "2", "--warmup", "1", "--dist-backend", "gloo"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=280) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [l for l in outs[0][0].splitlines() if l.strip()]
    assert len(lines) == 1 and not outs[1][0].strip()
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["config"]["packets_per_step_node"] == 16384
    assert line["ep_owned"]["rounds_per_step"][0] >= 2 and line["ep_owned"]["cross_rank_deliveries_per_step"] > 0


def test_family_oracle_equals_sequential():
    """test_config5_bench_regime's oracle: config 5's IPv4 and IPv6 packets as two batches
    on two datapaths (tests/harness.FamilyOracle, the split bench.py runs on the GPU) give
    one sequential run's outputs, CT4 / CT6 tables, summed policy counters and metrics,
    over two fresh steps."""
    import bench
    w = synth.config5(1 << 13, n_svc=400, n_ep=64, n_remote=256, seed=97)
    parts, where = bench.split_families(w)
    dp, om = H.oracle_dp(w)
    fo = H.FamilyOracle(w)
    for v in (1, 2):
        f = H.apply_variant(w.frames, *synth.port_variant(w, v))
        ref = dp.lxc_egress(f, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + v)
        host = [np.ascontiguousarray(f[np.nonzero(where[:, 0] == k)[0], :s]) for k, s in ((0, 64), (1, 128))]
        got = fo.lxc_egress(parts, host, w.now + v)
        for k in (0, 1):
            idx = np.nonzero(where[:, 0] == k)[0]
            for f_ in ("ret", "reason", "identity", "ct", "proxy", "nl", "nu"):
                assert (getattr(got[k], f_) == getattr(ref, f_)[idx]).all(), (v, k, f_)
        assert (fo.metrics() == dp.metrics()).all()
        assert (fo.policy_rows() == H.sorted_rows(*om["policy"].dump())).all()
        for name in ("ct4", "ct6"):
            assert fo.digest(name) == om[name].digest(), name
    assert sum(int((getattr(g, "ct") == 0).sum()) for g in got) > 0
