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
