"""Config 5 parity: the from-container egress path (bpf_lxc.c handle_ingress ->
handle_ipv4_from_lxc / ipv6_l3_from_lxc with lb4/lb6 services, egress conntrack and
policy, local delivery into the destination's ipv{4,6}_policy), HIP path via the
C-ABI against the CPU oracle, bit-exact: per-packet verdicts, drop reasons,
destination identities, CT results, proxy ports and lookup/write accounting; the
CT4 and CT6 tables; policy counters; cilium_metrics."""
import numpy as np
import pytest

from cilium_amd import synth
from tests import harness as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

FIELDS = ("ret", "reason", "identity", "ct", "proxy", "nl", "nu")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


def run_egress(ctx, w, dev, lo, hi, now, events=True):
    f, l, _ = H.to_dev(w, dev, lo, hi)
    src, fh = H.egress_inputs(w, dev, lo, hi)
    out = H.dev_out(hi - lo, dev)
    if events:
        out["frames_out"] = torch.zeros(f.shape, dtype=torch.uint8, device=dev)
    ctx.lxc_egress(f, l, out, now, src_ep=src, flow_hash=fh)
    return H.host_out(out)


def same_table(pm, om, name):
    pk, pv = pm[name].dump()
    ok, ov = om[name].dump()
    assert len(pk) == len(ok), (name, len(pk), len(ok))
    if len(ok):
        assert (H.sorted_rows(pk, pv) == H.sorted_rows(ok, ov)).all(), name


def check_egress(w, dev, batches, rounds=2, trace_agg=0, events=True):
    from tests.test_gpu_parity import same_frames, same_notifications, same_traces
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    if events:
        ctx.notify_attach(w.n)
        dp.notify_attach(w.n)
        ctx.trace_attach(3 * w.n, trace_agg)
        dp.trace_attach(3 * w.n, trace_agg)
    traces = []
    cuts = np.linspace(0, w.n, batches + 1).astype(int)
    for rnd in range(rounds):
        now = w.now + rnd * 3
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            o = run_egress(ctx, w, dev, lo, hi, now, events)
            ref = dp.lxc_egress(w.frames[lo:hi], w.length[lo:hi], w.extra["src_ep"][lo:hi],
                                w.extra["flow_hash"][lo:hi], now=now, frames_out=events)
            for k in FIELDS:
                bad = np.nonzero(o[k] != getattr(ref, k))[0]
                if len(bad):
                    v6 = w.extra["v6"][lo:hi][bad]
                    print("MISMATCH", k, "n", len(bad), "v6 frac", v6.mean(), "gpu ret/reason",
                          o["ret"][bad[:12]], o["reason"][bad[:12]], "ref", ref.ret[bad[:12]], ref.reason[bad[:12]],
                          "ct", o["ct"][bad[:12]], ref.ct[bad[:12]], "nl", o["nl"][bad[:12]], ref.nl[bad[:12]])
                assert len(bad) == 0, (k, rnd, lo, bad[:5], o[k][bad[:5]], getattr(ref, k)[bad[:5]])
            if not events:
                continue
            assert same_notifications(ctx, dp) == int((o["reason"] != 0).sum())   # one record per drop
            traces.append(same_traces(ctx, dp, ref.ret))
            same_frames(o["frames_out"], ref.frames_out, w.frames[lo:hi])
    if events:
        tr = np.concatenate(traces)
        assert (tr["subtype"] >= 5).any() == (trace_agg == 0)                # FROM_LXC hidden at >= 1
    assert (ctx.metrics() == dp.metrics()).all()
    for name in ("ct4", "ct6", "policy"):
        same_table(pm, om, name)
    ctx.close()
    return dp


def test_config5_dual_stack(dev):
    w = synth.config5(1 << 15, n_svc=2000, n_ep=256, n_remote=1024)
    check_egress(w, dev, batches=3)


def test_config5_plain_instances(dev):
    """No rings, no frames: the kernel instances the bench runs."""
    w = synth.config5(1 << 15, n_svc=2000, n_ep=256, n_remote=1024, seed=23)
    check_egress(w, dev, batches=2, events=False)


def test_config5_v4_records_64(dev):
    w = synth.config5(1 << 14, n_svc=1000, n_ep=128, n_remote=512, family=4, seed=51)
    assert w.frames.shape[1] == 64
    check_egress(w, dev, batches=2)


def test_config5_hot_flows(dev):
    # few flows and services with few backends: large groups, loopback services,
    # replies through rev-NAT, FIN/RST/SYN mixes in one batch
    w = synth.config5(1 << 14, n_svc=40, n_ep=8, n_remote=16, n_flows=64, seed=52, odd_frac=5.0)
    check_egress(w, dev, batches=2, rounds=3)


def test_config5_chunked(dev, monkeypatch):
    monkeypatch.setenv("CV_MAX_CHUNK", "5003")
    w = synth.config5(1 << 14, n_svc=500, n_ep=64, n_remote=128, seed=53)
    check_egress(w, dev, batches=1)


def test_config5_drop_all(dev):
    w = synth.config5(1 << 12, n_svc=200, n_ep=32, n_remote=64, seed=54)
    dp, om = H.oracle_dp(w, flags=H_flags(drop_all=True))
    ctx, pm = H.product_ctx(w, flags=H_flags(drop_all=True))
    o = run_egress(ctx, w, dev, 0, w.n, w.now)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    for k in FIELDS:
        assert (o[k] == getattr(ref, k)).all(), k
    assert (ctx.metrics() == dp.metrics()).all()
    ctx.close()


def H_flags(drop_all=False):
    from cilium_amd import lib
    return lib.F_DEFAULT | (lib.F_DROP_ALL if drop_all else 0)


def test_config5_v6_only(dev):
    w = synth.config5(1 << 13, n_svc=500, n_ep=64, n_remote=128, family=6, seed=55)
    check_egress(w, dev, batches=1, rounds=1)


def test_config5_v4_records_128(dev):
    w = synth.config5(1 << 13, n_svc=500, n_ep=64, n_remote=128, family=4, stride=128, seed=56)
    check_egress(w, dev, batches=1, rounds=1)


def nat_reader_workload():
    """A config-5 batch plus packets that read the NATed tuples service creates write:
    a non-loopback service create writes the self-pair key (backend, backend, flow
    ports); a backend sending to its own address with those ports (both port orders)
    looks it up later in the same batch.  The batch parallelism must order that reader
    after the writer (k_egress_nat: port-qualified self-pair nodes)."""
    w = synth.config5(1 << 13, n_svc=200, n_ep=64, n_remote=128, family=4, seed=61, vip_frac=0.9)
    dp, om = H.oracle_dp(w)
    dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    keys, _ = om["ct4"].dump()
    da = np.ascontiguousarray(keys[:, 0:4]).view("<u4").ravel()
    sa = np.ascontiguousarray(keys[:, 4:8]).view("<u4").ravel()
    fsa = np.ascontiguousarray(w.frames[:, 26:30]).view("<u4").ravel()
    v4ok = (w.frames[:, 12] == 8) & (w.frames[:, 13] == 0)
    readers = []
    for r in np.nonzero((da == sa) & np.isin(keys[:, 12], (6, 17)))[0]:
        q = np.nonzero(v4ok & (fsa == da[r]))[0]
        if not len(q):
            continue
        for ports in (keys[r, 8:12], np.concatenate([keys[r, 10:12], keys[r, 8:10]])):
            f = w.frames[q[0]].copy()
            f[30:34] = keys[r, 0:4]                               # daddr = the backend itself
            f[23] = keys[r, 12]
            f[34:38] = ports
            readers.append((f, q[0]))
        if len(readers) >= 64:
            break
    assert readers, "no NAT tuples in the batch"
    idx = np.array([q for _, q in readers])
    w.frames = np.concatenate([w.frames, np.stack([f for f, _ in readers])])
    w.length = np.concatenate([w.length, w.length[idx]])
    for k in ("src_ep", "flow_hash", "v6", "kind", "reply"):
        if k in w.extra:
            w.extra[k] = np.concatenate([w.extra[k], w.extra[k][idx]])
    w.mark = np.concatenate([w.mark, w.mark[idx]])
    return w, len(readers)


def test_config5_nat_tuple_readers(dev):
    w, nr = nat_reader_workload()
    dp, _ = H.oracle_dp(w)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    assert (ref.ct[-nr:] != 0).any(), "no crafted packet reads a NAT tuple"
    check_egress(w, dev, batches=1, rounds=1)


def test_config5_short_l4_checksum_fields(dev):
    """Packets whose L4 checksum field lies past the packet end (DROP_CSUM_L4 from the
    lb4_xlate / rev-NAT checksum helpers) or past the 64-B record (E_TRUNC)."""
    w = synth.config5(1 << 13, n_svc=200, n_ep=64, n_remote=128, family=4, seed=71)
    s = synth.Stream(5)
    tcp = (w.frames[:, 23] == 6) & (s.frac(w.n) < 0.3)
    w.length[tcp] = s.randint(int(tcp.sum()), 38, 52).astype(np.uint32)      # check @50 not in the packet
    udp = (w.frames[:, 23] == 17) & (s.frac(w.n) < 0.3)
    w.length[udp] = s.randint(int(udp.sum()), 38, 42).astype(np.uint32)      # check @40
    dp = check_egress(w, dev, batches=1, rounds=2)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + 9)
    assert (ref.ret == -154).any() or (ref.reason == -154).any()


def test_config5_v6_short_l4_checksum_fields(dev):
    """IPv6 packets whose L4 checksum field (TCP @16, UDP @6, ICMPv6 @2 of the L4
    header) lies past the packet end: DROP_CSUM_L4 from lb6_xlate, __lb6_rev_nat and the
    rev-NAT index zeroing of ipv6_policy; frames of the rest byte-exact."""
    w = synth.config5(1 << 13, n_svc=200, n_ep=64, n_remote=128, family=6, seed=73)
    s = synth.Stream(6)
    v6 = (w.frames[:, 12] == 0x86) & (w.frames[:, 13] == 0xDD)
    tcp = v6 & (w.frames[:, 20] == 6) & (s.frac(w.n) < 0.3)
    w.length[tcp] = s.randint(int(tcp.sum()), 58, 72).astype(np.uint32)      # check @70 not in the packet
    udp = v6 & (w.frames[:, 20] == 17) & (s.frac(w.n) < 0.3)
    w.length[udp] = s.randint(int(udp.sum()), 58, 62).astype(np.uint32)      # check @60
    dp = check_egress(w, dev, batches=1, rounds=2)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now + 9)
    assert (ref.ret == -154).any() or (ref.reason == -154).any()


@pytest.mark.parametrize("agg", [1, 3])
def test_config5_traces_aggregated(dev, agg):
    """send_trace_notify at MONITOR_AGGREGATION lowest (FROM_* hidden) and medium (only
    the steps whose CT lookup asked for a report: new flows, new TCP flags, or
    CT_REPORT_INTERVAL elapsed; rounds 3 s apart cross the 5 s interval)."""
    w = synth.config5(1 << 14, n_svc=500, n_ep=128, n_remote=512, seed=91)
    check_egress(w, dev, batches=2, rounds=3, trace_agg=agg)


def test_empty_batches(dev):
    """n = 0 at every batch entry point: no launch, no error, no state change; the next
    real batch still matches the oracle."""
    w = synth.config5(1 << 12, n_svc=200, n_ep=32, n_remote=64, seed=57)
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    f, l, m = H.to_dev(w, dev, 0, 0)
    src, fh = H.egress_inputs(w, dev, 0, 0)
    out = H.dev_out(0, dev)
    ctx.lxc_egress(f, l, out, w.now, src_ep=src, flow_hash=fh)
    ctx.netdev_ingress(f, l, out, w.now, mark=m)
    ctx.policy_ingress(0, f, l, out, mark=m)
    ctx.xdp_prefilter(f, l, out)
    torch.cuda.synchronize()
    assert not ctx.metrics().any()
    assert len(pm["ct4"].dump()[0]) == 0
    o = run_egress(ctx, w, dev, 0, w.n, w.now)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
    for k in FIELDS:
        assert (o[k] == getattr(ref, k)).all(), k
    assert (ctx.metrics() == dp.metrics()).all()
    same_table(pm, om, "ct4")
    ctx.close()


def _v6_ext_chains(w, seed, frac=0.5):
    """Rewrite a fraction of the IPv6 records with extension-header chains in front of
    their L4 header: 0-5 headers from HOPOPTS / ROUTING / DSTOPTS / AUTH (sizes as
    ipv6_hdrlen computes them, bpf/lib/ipv6.h:61-98, including the AUTH-length quirk),
    now and then FRAGMENT or NONE, chains that run past skb->len or past the record."""
    s = synth.Stream(seed)
    f, ln = w.frames, w.length
    stride = f.shape[1]
    rows = np.nonzero((f[:, 12] == 0x86) & (f[:, 13] == 0xDD) & (s.frac(len(ln)) < frac))[0]
    for i in rows:
        nh0 = int(f[i, 20])
        l4off = 62 if nh0 == 0 else 54
        proto = int(f[i, 54]) if nh0 == 0 else nh0
        l4 = f[i, l4off:l4off + 24].copy()
        k = int(s.randint(1, 0, 6)[0])
        types = [int(t) for t in np.array([0, 43, 60, 51, 51, 43, 44, 59])[s.choice(k, 8)]] if k else []
        chain = bytearray()
        for j, t in enumerate(types):
            nxt = types[j + 1] if j + 1 < k else proto
            h = int(s.randint(1, 0, 3)[0])
            size = (h + 2) * 4 if nxt == 51 else (h + 1) * 8
            hdr = bytearray(size)
            hdr[0], hdr[1] = nxt, h
            chain += hdr
        body = bytes(chain) + l4.tobytes()
        f[i, 54:] = 0
        n = min(len(body), stride - 54)
        f[i, 54:54 + n] = np.frombuffer(body[:n], np.uint8)
        f[i, 20] = types[0] if k else proto
        f[i, 18:20] = synth.be16_bytes(np.array([len(body) - 4], np.uint16))
        r = s.frac(1)[0]
        ln[i] = 54 + len(body) if r < 0.6 else (90 if r < 0.8 else 54 + len(chain) + 2)


def test_config5_v6_extension_headers(dev):
    w = synth.config5(1 << 13, n_svc=300, n_ep=48, n_remote=96, family=6, seed=58)
    _v6_ext_chains(w, 0xE7)
    check_egress(w, dev, batches=2)


def test_ct_capacity_egress(dev):
    """Egress CT4 / CT6 maps reaching max_entries inside a batch: service creates,
    connection creates with their NAT tuples and the delivery's ingress creates fail
    past the limit exactly where the sequential oracle's do."""
    w = synth.config5(1 << 12, n_svc=2000, n_ep=256, n_remote=512, ct_max=1500)
    dp = check_egress(w, dev, batches=2, rounds=1)
    assert dp.metrics()[155, 2, 0] + dp.metrics()[155, 1, 0] > 0       # DROP_CT_CREATE_FAILED happened


def test_ct_capacity_egress_admitted(dev, monkeypatch):
    """A 2^20-packet config-5 batch whose creates cross max_entries in CT4 (about 2/3 in)
    and CT6 (about 3/4 in), at full width (cv_ctx.cpp lxc_admitted: the pipeline runs with
    per-packet create budgets until the budget scan says every packet got the sequential
    run's creates); then a batch into the full maps after the agent removed a third of the
    ingress L4 policy entries, so denied established flows are deleted and later packets'
    creates take the room, in packet order.  Verdicts, tables, counters, metrics exact."""
    monkeypatch.setenv("CV_ADMIT_STATS", "1")
    w = synth.config5(1 << 20, n_svc=20000, n_ep=1024, n_remote=4096, seed=81, ct_max=300_000)
    dp, om = H.oracle_dp(w)
    ctx, pm = H.product_ctx(w)
    for rnd in (0, 1):
        if rnd == 1:
            keys = w.maps["policy"].keys
            for k in keys[(keys[:, 6] != 0) & (keys[:, 7] == 0)][::3]:           # ingress, L4
                assert pm["policy"].delete(k.tobytes()) == 0 == om["policy"].delete(k.tobytes())
        now = w.now + 3 * rnd
        o = run_egress(ctx, w, dev, 0, w.n, now, events=False)
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=now)
        for k in FIELDS:
            bad = np.nonzero(o[k] != getattr(ref, k))[0]
            assert len(bad) == 0, (rnd, k, len(bad), bad[:5], o[k][bad[:5]], getattr(ref, k)[bad[:5]])
        assert (ctx.metrics() == dp.metrics()).all(), rnd
        for name in ("ct4", "ct6", "policy"):
            same_table(pm, om, name)
        assert len(pm["ct4"]) == len(om["ct4"]) and len(pm["ct6"]) == len(om["ct6"])
    m = dp.metrics()
    assert m[155, 2, 0] + m[155, 1, 0] > 100_000                           # DROP_CT_CREATE_FAILED
    assert len(om["ct4"]) == len(om["ct6"]) == 300_000
    ctx.close()


def test_config5_elephant_flows(dev):
    """Four flows carry a 2^16-packet batch: groups of thousands of members, past the
    grouping's LDS sort (k_gbin_group: the bin split by sub-bins and the elephant's
    members ordered by packet through the tile bitmaps), in position lists."""
    w = synth.config5(1 << 16, n_svc=40, n_ep=8, n_remote=16, n_flows=4, seed=59)
    check_egress(w, dev, batches=1, rounds=2)


def test_ct_capacity_egress_admission_fallback(dev, monkeypatch):
    """An egress launch whose admission finds no fixed point within its pass limit
    (forced here: one pass, which a batch crossing max_entries cannot settle in) puts the
    maps back as they were and runs the chunk again in planned launches, guarded next to
    the limit: still the sequential run's answer."""
    monkeypatch.setenv("CV_EADM_MAX_PASSES", "1")
    w = synth.config5(1 << 12, n_svc=2000, n_ep=256, n_remote=512, ct_max=1500, seed=83)
    dp = check_egress(w, dev, batches=2, rounds=1)
    assert dp.metrics()[155, 2, 0] + dp.metrics()[155, 1, 0] > 0       # DROP_CT_CREATE_FAILED happened


def test_acct_split_counts(dev):
    """CV_F_ACCT_SPLIT (bench.py's HBM-resident split): nl / nu count every conntrack lookup
    / write ACCT_CT_UNIT and every other lookup / write 1, equal to the oracle's under the
    same split -- config 5 (service, egress and delivery conntrack) and config 3 (netdev)."""
    from cilium_amd import lib
    from oracle import oracle as O
    from tests.test_gpu_parity import run_ingress
    try:
        O.set_acct_split(True)
        w = synth.config5(1 << 15, n_svc=1000, n_ep=128, n_remote=512, seed=95)
        dp, om = H.oracle_dp(w)
        ctx, pm = H.product_ctx(w, flags=lib.F_DEFAULT | lib.F_ACCT_SPLIT)
        o = run_egress(ctx, w, dev, 0, w.n, w.now, events=False)
        ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now)
        for k in ("ret", "nl", "nu"):
            assert (o[k] == getattr(ref, k)).all(), k
        assert (o["nl"] >= lib.ACCT_CT_UNIT).sum() > w.n // 2 and (o["nl"] % lib.ACCT_CT_UNIT).sum() > 0
        ctx.close()
        w = synth.config3(1 << 15, 1 << 13, n_ep=64, n_cidrs=1024, n_ids=100, seed=96)
        dp, om = H.oracle_dp(w)
        ctx, pm = H.product_ctx(w, flags=lib.F_DEFAULT | lib.F_ACCT_SPLIT)
        o = run_ingress(ctx, w, dev, 0, w.n, events=False)
        ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now)
        for k in ("ret", "nl", "nu"):
            assert (o[k] == getattr(ref, k)).all(), k
        assert (o["nl"] >= lib.ACCT_CT_UNIT).sum() > w.n // 4
        ctx.close()
    finally:
        O.set_acct_split(False)
