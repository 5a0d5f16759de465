"""Seed sweep of the HIP path against the oracle: the parity tests elsewhere each pin one
seed; these draw several more batches of configs 3 and 5 with the rare cases made common
(odd frames, TTL 1, unknown protocols, hop-by-hop headers, ARP and neighbour solicitations
ten times as often as the bench's mix) and other flow / service mixes.  Every output, the
drop and trace records, the rewritten frames, the counters and every table, bit-exact."""
import numpy as np
import pytest

from cilium_amd import synth
from tests.test_gpu_egress import check_egress
from tests.test_gpu_parity import check_ingress

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


@pytest.mark.parametrize("seed,vip,reply,kw", [
    (101, 0.7, 0.2, {}), (102, 0.4, 0.5, {}), (103, 0.9, 0.05, {}), (104, 0.2, 0.8, {}),
    (105, 0.7, 0.3, {"family": 4}), (106, 0.7, 0.3, {"family": 6}), (107, 0.6, 0.4, {"ep_zipf": 0.9}),
    (108, 0.8, 0.3, {"n": 1 << 17, "n_flows": 1 << 12})])
def test_config5_seed_sweep(dev, seed, vip, reply, kw):
    kw = dict(kw)
    n = kw.pop("n", 1 << 15)
    w = synth.config5(n, seed=seed, n_svc=1500, n_ep=192, n_remote=640, vip_frac=vip, reply_frac=reply,
                      odd_frac=10.0, **kw)
    check_egress(w, dev, batches=3)


@pytest.mark.parametrize("seed,v6,zipf,flows,n", [
    (201, 0.3, None, 1 << 12, 1 << 15), (202, 0.0, 0.9, 1 << 12, 1 << 15), (203, 0.5, 1.1, 1 << 12, 1 << 15),
    (204, 0.2, None, 1 << 12, 1 << 15), (205, 0.0, None, 256, 1 << 15), (206, 0.4, 0.6, 1 << 14, 1 << 17),
    (207, 1.0, None, 1 << 12, 1 << 15), (208, 0.1, 1.3, 1 << 10, 1 << 16)])
def test_config3_seed_sweep(dev, seed, v6, zipf, flows, n):
    w = synth.config3(n, flows, seed=seed, n_ep=128, n_cidrs=2048, n_ids=300, v6_frac=v6, zipf=zipf, ttl_low=0.01)
    check_ingress(w, dev, batches=3)


@pytest.mark.parametrize("seed,zipf,full,steps", [(301, 0.6, 6, 3), (302, 1.0, 20, 2), (303, None, 40, 2),
                                                  (304, 0.8, 12, 3)])
def test_config5_ct_local_seed_sweep(dev, seed, zipf, full, steps):
    """ConntrackLocal egress next to max_entries over several seeds: per-endpoint CT4 / CT6
    maps sized so the `full` busiest fill, bench-shaped steps (synth.port_variant), the
    admitted launches (two budgets per packet, passes undone from the slot log) exact."""
    import copy
    from tests import ep_shard as E
    from tests import harness as H
    from tests.test_gpu_egress import run_egress
    from tests.test_gpu_ep_node import per_endpoint_ctx
    from tests.test_gpu_ep_maps import EGR, _check_fields
    kw = dict(n_svc=2000, n_ep=192, n_remote=640, seed=seed, ep_zipf=zipf)
    n = 1 << 16
    w = synth.config5(n, ct_max=1 << 20, **kw)
    dp0, m0 = E.per_endpoint_dp(w)
    dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
    cap = int(sizes[-full])
    w = synth.config5(n, ct_max=cap, **kw)
    dp, om = E.per_endpoint_dp(w)
    ctx, pm = per_endpoint_ctx(w)
    for v in range(1, steps + 1):
        wv = copy.copy(w)
        wv.frames = H.apply_variant(w.frames, *synth.port_variant(w, v))
        o = run_egress(ctx, wv, dev, 0, w.n, w.now + v, events=False)
        ref = dp.lxc_egress(wv.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + v)
        _check_fields(o, ref, EGR, v)
        assert (ctx.metrics() == dp.metrics()).all(), v
    for fam in ("ct4", "ct6"):
        for e, (a, b) in enumerate(zip(pm[fam], om[fam])):
            ak, av = a.dump()
            bk, bv = b.dump()
            assert len(ak) == len(bk) and (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all(), (fam, e)
    ok, ov = om["policy"].dump()
    pk, pv = pm["policy"].dump()
    assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all()
    ctx.close()


@pytest.mark.parametrize("seed,zipf,full", [(401, 1.1, 20), (402, 0.8, 8), (403, 1.3, 40)])
def test_config3_ct_local_seed_sweep(dev, seed, zipf, full):
    """ConntrackLocal ingress next to max_entries over several seeds: per-endpoint CT4 maps
    with the `full` busiest full from the start, two batches, admitted and exact."""
    from tests import harness as H
    from tests.test_gpu_ep_maps import ING, _check_fields
    from tests.test_gpu_parity import run_ingress
    w = synth.config3(1 << 16, 1 << 14, n_ep=128, n_cidrs=2048, n_ids=300, seed=seed, ep_zipf=zipf)
    per = synth.per_endpoint_ct(w, 1 << 20)
    counts = np.array(sorted(len(s) for s in per))
    cap = int(counts[-full])
    per = synth.per_endpoint_ct(w, cap)
    dp, om = H.oracle_dp(w, ct_per_ep=per)
    ctx, pm = H.product_ctx(w, ct_per_ep=per)
    for r in range(2):
        wr = synth.Workload(w.name, w.maps, w.frames, w.length, w.mark, w.endpoints, now=w.now + r, extra=w.extra)
        o = run_ingress(ctx, wr, dev, 0, w.n, events=False)
        ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now + r)
        _check_fields(o, ref, ING, r)
        assert (ctx.metrics() == dp.metrics()).all(), r
    for a, b in zip(pm["ct4_ep"], om["ct4_ep"]):
        ak, av = a.dump()
        bk, bv = b.dump()
        assert len(ak) == len(bk) and (H.sorted_rows(ak, av) == H.sorted_rows(bk, bv)).all()
    assert dp.metrics()[155, 1, 0] > 0                           # DROP_CT_CREATE_FAILED in the full maps
    ctx.close()


@pytest.mark.parametrize("seed,frac", [(0xF1, 0.0), (0xF2, 0.25), (0xF3, 0.5), (0xF4, 0.75)])
def test_endpoint_owned_seed_sweep(dev, seed, frac):
    """The endpoint-owned node (the native scheduler driving the HIP split / deliver
    launches) over several seeds, with none, a quarter, half or three quarters of the
    per-endpoint maps filling within the batch: the sequential per-endpoint oracle's
    every output, table, counter and metric."""
    from tests import ep_shard as E
    from tests.test_gpu_ep_node import _check, _rank_run
    kw = dict(n_svc=120, n_ep=24, n_remote=32, seed=seed, vip_frac=0.5)
    w = synth.config5(1 << 12, ct_max=1 << 16, **kw)
    if frac:
        dp0, m0 = E.per_endpoint_dp(w)
        dp0.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
        sizes = np.array(sorted(max(len(a), len(b)) for a, b in zip(m0["ct4"], m0["ct6"])))
        w = synth.config5(1 << 12, ct_max=int(sizes[int(len(sizes) * (1 - frac))]), **kw)
    _check(w, [_rank_run(w, 0, 1, dev)])
