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


@pytest.mark.parametrize("seed,vip,reply", [(101, 0.7, 0.2), (102, 0.4, 0.5), (103, 0.9, 0.05), (104, 0.2, 0.8)])
def test_config5_seed_sweep(dev, seed, vip, reply):
    w = synth.config5(1 << 15, seed=seed, n_svc=1500, n_ep=192, n_remote=640, vip_frac=vip, reply_frac=reply,
                      odd_frac=10.0)
    check_egress(w, dev, batches=3)


@pytest.mark.parametrize("seed,v6,zipf", [(201, 0.3, None), (202, 0.0, 0.9), (203, 0.5, 1.1), (204, 0.2, None)])
def test_config3_seed_sweep(dev, seed, v6, zipf):
    w = synth.config3(1 << 15, 1 << 12, seed=seed, n_ep=128, n_cidrs=2048, n_ids=300, v6_frac=v6, zipf=zipf,
                      ttl_low=0.01)
    check_ingress(w, dev, batches=3)
