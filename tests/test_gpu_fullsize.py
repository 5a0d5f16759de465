"""Parity at BASELINE.json's table sizes: the HIP path
(through the C-ABI) against the CPU oracle on the same seeded inputs.

* config 3: the full 16M-flow conntrack table (33.6M entries with the ICMP-RELATED
  twins), the 100k-CIDR ipcache and 10k-identity policy, 4096 endpoints, a 2^19-packet
  batch the oracle runs in seconds: every per-packet output, cilium_metrics, the
  policy counters, and the whole CT table after the batch through an
  order-independent digest (tests/harness.table_digest = the oracle's or_map_digest);
* config 4: one rank's part of the node-wide flow set (bench.py at N > 1, two ranks'
  shards here, each against its own oracle: shards share no conntrack state);
* config 5: the 50k-service dual-stack egress tables.
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
