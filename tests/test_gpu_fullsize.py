"""Parity at BASELINE.json's table sizes: the HIP path
(through the C-ABI) against the CPU oracle on the same seeded inputs.

* config 3: the full 16M-flow conntrack table (33.6M entries with the ICMP-RELATED
  twins), the 100k-CIDR ipcache and 10k-identity policy, 4096 endpoints, a 2^19-packet
  batch the oracle runs in seconds: every per-packet output, cilium_metrics, the
  policy counters, and the whole CT table after the batch through an
  order-independent digest (tests/harness.table_digest = the oracle's or_map_digest);
* config 4: one rank's part of the node-wide flow set (bench.py at N > 1, two ranks'
  shards here, each against its own oracle: shards share no conntrack state);
* config 5: the 50k-service dual-stack egress tables;
* bench.py's own timed regime (round 3): two consecutive fresh 2^24-packet config-3
  steps on the 16M-flow table with the CT sized as bench.py sizes it, and rank 0 of 8's
  config-4 shard at BASELINE size (16M flows), against the address-pair-sharded oracle
  (tests/harness.ShardedOracle): every per-packet output, metrics, the node's policy
  counters and the CT digest after each step.
"""
import numpy as np
import pytest

from cilium_amd import shard, synth
from tests import harness as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

FIELDS = ("xdp", "ret", "identity", "ct", "proxy", "nl", "nu", "reason")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


def _ingress_vs_oracle(w, dev, n):
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    f, l, m = H.to_dev(w, dev, 0, n)
    out = H.dev_out(n, dev)
    ctx.netdev_ingress(f, l, out, w.now, mark=m)
    o = H.host_out(out)
    ref = dp.netdev_ingress(w.frames[:n], w.length[:n], w.mark[:n], now=w.now)
    for k in FIELDS:
        bad = np.nonzero(o[k] != getattr(ref, k))[0]
        assert len(bad) == 0, (k, bad[:5], o[k][bad[:5]], getattr(ref, k)[bad[:5]])
    assert (ctx.metrics() == dp.metrics()).all()
    pk, pv = pm["policy"].dump()
    ok, ov = om["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    return ctx, pm, om, o


def test_config3_full_table(dev):
    n = 1 << 19
    w = synth.config3(n, 1 << 24)
    ctx, pm, om, o = _ingress_vs_oracle(w, dev, n)
    ck, cv = pm["ct4"].dump()
    want = om["ct4"].digest()
    assert want[0] > 33_000_000                                   # the full table, twins included
    assert H.table_digest(ck, cv) == want
    assert (o["ct"] == 0).sum() > n // 20                         # the batch created entries
    ctx.close()


def test_config4_rank_shards(dev):
    world = 2
    seen = None
    for rank in range(world):
        w = synth.config3(1 << 18, 1 << 21, seed=0xC1A00004, shard=(rank, world))
        assert (shard.flow_shard(w.frames, w.length, world) == rank).all()
        ctx, pm, om, _ = _ingress_vs_oracle(w, dev, w.n)
        ck, cv = pm["ct4"].dump()
        assert H.table_digest(ck, cv) == om["ct4"].digest()
        assert (shard.ct4_shard(ck, world) == rank).all()          # creates stay on their rank
        keys = set(map(bytes, ck[::97]))
        if seen is not None:
            assert not (keys & seen)
        seen = keys
        ctx.close()


@pytest.fixture
def say(capsys):
    """progress lines past pytest's capture (a minutes-long test stays visibly alive)"""
    import time
    t0 = time.time()

    def f(msg):
        with capsys.disabled():
            print(f"  [{time.time() - t0:6.1f}s] {msg}", flush=True)
    return f


def _bench_steps(w, dev, steps, say, threads, ct_check=None):
    """bench.py's timed regime on the device and on the address-pair-sharded oracle:
    step v = the batch with fresh client ports on its new flows (synth.port_variant),
    built on the device as bench.py builds it, `now + v`; after each step every
    per-packet output, cilium_metrics, the node's policy counters and the CT table
    digest against the oracle."""
    from cilium_amd import synth
    so = H.ShardedOracle(w, threads)
    say(f"oracle: {threads} address-pair shards loaded")
    ctx, pm = H.product_ctx(w)
    frames, length, mark = H.to_dev(w, dev)
    out = H.dev_out(w.n, dev)
    say("device tables compiled")
    for v in steps:
        rows, boff, ports = synth.port_variant(w, v)
        fv = frames.clone()
        r, o = torch.from_numpy(rows).to(dev), torch.from_numpy(boff).to(dev)
        fv[r, o] = torch.from_numpy((ports >> 8).astype(np.uint8)).to(dev)
        fv[r, o + 1] = torch.from_numpy((ports & 0xFF).astype(np.uint8)).to(dev)
        ctx.netdev_ingress(fv, length, out, w.now + v, mark=mark)
        got = H.host_out(out)
        del fv
        ref, el = so.netdev_ingress(H.apply_variant(w.frames, rows, boff, ports), now=w.now + v)
        say(f"step {v}: device done, oracle {el:.1f}s")
        for k in FIELDS:
            bad = np.nonzero(got[k] != getattr(ref, k))[0]
            assert len(bad) == 0, (v, k, bad[:5], got[k][bad[:5]], getattr(ref, k)[bad[:5]])
        assert (ctx.metrics() == so.metrics()).all()
        pk, pv = pm["policy"].dump()
        assert (H.sorted_rows(pk, pv) == so.policy_rows()).all()
        want = so.digest("ct4")
        ck, cv = pm["ct4"].dump()
        assert H.table_digest(ck, cv) == want, v
        if ct_check is not None:
            assert ct_check(ck)
        say(f"step {v}: outputs, metrics, policy counters and the {want[0]}-entry CT bit-exact "
            f"({int((got['ct'] == 0).sum())} CT_NEW)")
        del ck, cv
    ctx.close()
    return so


def test_config3_bench_regime(dev, say):
    """The regime bench.py times (verdict r02 item 1): the 2^24-packet config-3 batch
    on the 16M-flow table with the CT sized by bench.size_conntrack for a default run,
    two consecutive fresh steps (2.58M creates each), bit-exact against the oracle."""
    import bench
    w = bench.make_workload("config3", 1 << 24, 0, 1)
    bench.size_conntrack("config3", w, passes=3 + 20 + 1)
    say(f"workload: {w.n} packets, {len(w.maps['ct4'].keys)} CT entries, max_entries {w.maps['ct4'].max_entries}")
    _bench_steps(w, dev, (1, 2), say, bench.allowed_cpus())


def test_config4_rank_shard_full_size(dev, say):
    """Config 4 at BASELINE's size: rank 0 of 8's part of the 128M-flow node-wide set
    (16M flows, 33.5M CT entries) and packets of its own address pairs, two fresh
    steps bit-exact against the oracle; every CT entry stays on its rank."""
    import bench
    w = synth.config3(1 << 22, 1 << 24, seed=0xC1A00004, shard=(0, 8))
    assert (shard.flow_shard(w.frames, w.length, 8) == 0).all()
    assert (shard.ct4_shard(w.maps["ct4"].keys, 8) == 0).all()
    bench.size_conntrack("config4", w, passes=3)
    say(f"workload: rank 0 of 8, {w.n} packets, {len(w.maps['ct4'].keys)} CT entries")
    _bench_steps(w, dev, (1, 2), say, bench.allowed_cpus(),
                 ct_check=lambda keys: (shard.ct4_shard(keys, 8) == 0).all())      # creates stay on the rank


def test_config5_full_services(dev):
    from tests.test_gpu_egress import run_egress
    w = synth.config5(1 << 17)                                    # 50k services, 4096 endpoints
    assert len(w.maps["lb4_revnat"]) + len(w.maps["lb6_revnat"]) == 50_000    # services (v4 + v6)
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    o = run_egress(ctx, w, dev, 0, w.n, w.now, events=False)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    for k in ("ret", "reason", "identity", "ct", "proxy", "nl", "nu"):
        bad = np.nonzero(o[k] != getattr(ref, k))[0]
        assert len(bad) == 0, (k, bad[:5], o[k][bad[:5]], getattr(ref, k)[bad[:5]])
    assert (ctx.metrics() == dp.metrics()).all()
    for name in ("ct4", "ct6"):
        ck, cv = pm[name].dump()
        assert H.table_digest(ck, cv) == om[name].digest(), name
    ctx.close()


def test_config5_bench_regime(dev, say):
    """The config-5 regime bench.py times (verdict r04 item 1): the 2^24-packet dual-stack
    egress batch (50k services, 4096 endpoints) with the CT maps sized by
    bench.size_conntrack for a default run, split into its IPv4 (64-B) and IPv6 (128-B)
    launches, two consecutive fresh steps built on the device by bench.step_batch: every
    per-packet output, cilium_metrics, the policy counters and the CT4 / CT6 digests after
    each step, bit-exact against the oracle.  At this size the position lists, the
    continuation lanes and the binned groupings run at the bench's occupancy."""
    import bench
    w = bench.make_workload("config5", 1 << 24, 0, 1)
    bench.size_conntrack("config5", w, passes=3 + 20 + 1)
    parts, where = bench.split_families(w)
    say(f"workload: {w.n} packets ({len(parts[0]['length'])} v4, {len(parts[1]['length'])} v6), "
        f"CT max_entries {w.maps['ct4'].max_entries} / {w.maps['ct6'].max_entries}")
    fo = H.FamilyOracle(w)
    say("oracle: one datapath per family loaded")
    ctx, pm = H.product_ctx(w)
    dev_parts = [{k: bench.to_device(v, dev) for k, v in p.items()} for p in parts]
    base = [p["frames"] for p in dev_parts]
    say("device tables compiled")
    from cilium_amd import lib
    from oracle import oracle as O
    for v in (1, 2):
        split = v == 2                                 # (step 2: nl / nu with the conntrack share split out)
        ctx.set_flags(lib.F_DEFAULT | (lib.F_ACCT_SPLIT if split else 0))
        O.set_acct_split(split)
        fv = bench.step_batch("config5", w, v, base, where, dev)
        got = []
        for k, p in enumerate(dev_parts):
            out = H.dev_out(len(parts[k]["length"]), dev)
            del out["xdp"]
            ctx.lxc_egress(fv[k], p["length"], out, w.now + v, src_ep=p["src_ep"], flow_hash=p["flow_hash"])
            got.append(H.host_out(out))
        del fv
        rows, boff, ports = synth.port_variant(w, v)
        fr = H.apply_variant(w.frames, rows, boff, ports)
        host = [np.ascontiguousarray(fr[np.nonzero(where[:, 0] == k)[0], :s]) for k, s in ((0, 64), (1, 128))]
        del fr
        t0 = __import__("time").time()
        refs = fo.lxc_egress(parts, host, w.now + v)
        say(f"step {v}: device done, oracle {__import__('time').time() - t0:.1f}s")
        for k in (0, 1):
            for f in ("ret", "reason", "identity", "ct", "proxy", "nl", "nu"):
                bad = np.nonzero(got[k][f] != getattr(refs[k], f))[0]
                assert len(bad) == 0, (v, k, f, bad[:5], got[k][f][bad[:5]], getattr(refs[k], f)[bad[:5]])
        assert (ctx.metrics() == fo.metrics()).all(), v
        pk, pv = pm["policy"].dump()
        assert (H.sorted_rows(pk, pv) == fo.policy_rows()).all(), v
        for name in ("ct4", "ct6"):
            ck, cv = pm[name].dump()
            assert H.table_digest(ck, cv) == fo.digest(name), (v, name)
            del ck, cv
        news = sum(int((g["ct"] == 0).sum()) for g in got)
        say(f"step {v}: outputs, metrics, policy counters, CT4 {fo.digest('ct4')[0]} / CT6 {fo.digest('ct6')[0]} "
            f"entries bit-exact ({news} CT_NEW)" + (", nl / nu split (conntrack share) equal" if split else ""))
        if split:
            ctl = sum(int((g["nl"].astype(np.int64) // lib.ACCT_CT_UNIT).sum()) for g in got)
            assert ctl > w.n                           # (every IP packet probes its conntrack map at least once)
    O.set_acct_split(False)
    ctx.close()
