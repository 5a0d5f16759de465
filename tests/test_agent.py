"""The agent-side state machines of include/cilium_agent.h over the engine's map store:
the XDP prefilter's revisioned CIDR sets (pkg/policy/prefilter.go) and an endpoint's
policy-map sync (pkg/endpoint/endpoint.go:2524-2604).  The reference has no unit tests
for either; the expectations below restate the Go code's behaviour line by line (cited
per test).  CPU tests use a host-only context; the GPU test drives the XDP datapath
with CIDRs written through the prefilter and checks it against the oracle."""
import copy
import ipaddress
import struct

import pytest

from cilium_amd import lib, synth
from tests import harness as H


@pytest.fixture
def ctx():
    c = lib.Ctx(-1)
    yield c
    c.close()


def errno_of(excinfo):
    return excinfo.value.errno


# ------------------------------------------------------------------ prefilter
def test_prefilter_default_config(ctx):
    # NewPreFilter (prefilter.go:281-298): fix4 + fix6, revision 1; WriteConfig (:65-89)
    pf = lib.PreFilter(ctx)
    assert pf.map_handle(lib.PF_V4_FIX) >= 0 and pf.map_handle(lib.PF_V6_FIX) >= 0
    assert pf.map_handle(lib.PF_V4_DYN) == -1 and pf.map_handle(lib.PF_V6_DYN) == -1
    assert pf.dump() == ([], 1)
    assert pf.write_config() == (
        "#define CIDR4_HMAP_ELEMS 20971520\n#define CIDR4_LMAP_ELEMS 65536\n"
        "#define CIDR4_HMAP_NAME cilium_cidr_v4_fix\n#define CIDR4_LMAP_NAME .\n"
        "#define CIDR6_HMAP_NAME cilium_cidr_v6_fix\n#define CIDR6_LMAP_NAME .\n"
        "#define CIDR4_FILTER\n#define CIDR6_FILTER\n")
    pf.close()


def test_prefilter_insert_delete_revisions(ctx):
    pf = lib.PreFilter(ctx)
    pf.insert(1, ["1.2.3.4/32", "fd00::1/128"])                   # revision 1 -> 2
    cidrs, rev = pf.dump()
    assert rev == 2 and sorted(cidrs) == ["1.2.3.4/32", "fd00::1/128"]
    with pytest.raises(lib.CvError) as e:                         # Insert: stale revision (:131-133)
        pf.insert(1, ["5.6.7.8/32"])
    assert str(e.value).endswith("Latest revision is 2 not 1") or "Latest revision is 2 not 1" in str(e.value)
    # a CIDR without an enabled map stops the batch; the applied part is undone (:136-158)
    with pytest.raises(lib.CvError) as e:
        pf.insert(0, ["5.6.7.8/32", "10.0.0.0/8"])
    assert "No map enabled for CIDR string 10.0.0.0/8" in str(e.value)
    assert sorted(pf.dump()[0]) == ["1.2.3.4/32", "fd00::1/128"] and pf.dump()[1] == 2
    # Delete checks every CIDR before changing anything (:170-182)
    with pytest.raises(lib.CvError) as e:
        pf.delete(0, ["1.2.3.4/32", "9.9.9.9/32"])
    assert errno_of(e) == 2 and "No map entry for CIDR string 9.9.9.9/32" in str(e.value)
    assert len(pf.dump()[0]) == 2
    pf.delete(2, ["1.2.3.4/32"])
    assert pf.dump() == (["fd00::1/128"], 3)
    pf.close()


def test_prefilter_v6_fix_follows_fix4(ctx):
    # initOneMap creates the v6 fix map only when fix4 is enabled (prefilter.go:237)
    pf = lib.PreFilter(ctx, lib.PF_FIX6)
    assert pf.map_handle(lib.PF_V6_FIX) == -1
    with pytest.raises(lib.CvError) as e:
        pf.insert(0, ["fd00::1/128"])
    assert "No map enabled for CIDR string fd00::1/128" in str(e.value)
    assert "#define CIDR6_FILTER" in pf.write_config() and "CIDR6_HMAP_NAME .\n" in pf.write_config()
    pf.close()


def test_prefilter_dyn_maps_lpm_exists(ctx):
    pf = lib.PreFilter(ctx, lib.PF_DYN4 | lib.PF_FIX4 | lib.PF_DYN6 | lib.PF_FIX6)
    pf.insert(0, ["10.0.0.0/8", "192.168.1.0/24", "fd00:1::/32"])
    assert sorted(pf.dump()[0]) == ["10.0.0.0/8", "192.168.1.0/24", "fd00:1::/32"]
    cfg = pf.write_config()
    assert "#define CIDR4_LPM_PREFILTER\n" in cfg and "#define CIDR6_LPM_PREFILTER\n" in cfg
    # CIDRExists is a map lookup, an LPM match on the trie (cidrmap.go:108-113): a prefix
    # covered by 10.0.0.0/8 passes Delete's check, then DeleteCIDR (exact) fails and
    # nothing changes, revision included
    rev = pf.dump()[1]
    with pytest.raises(lib.CvError) as e:
        pf.delete(0, ["10.1.0.0/16"])
    assert errno_of(e) == 2 and "Error deleting CIDR string 10.1.0.0/16" in str(e.value)
    assert pf.dump()[1] == rev and len(pf.dump()[0]) == 3
    pf.close()


def test_prefilter_undo_on_full_map(ctx):
    # the 65537th dyn prefix overflows the 64k LPM map (maxLKeys): the whole batch is
    # undone (prefilter.go:154-158) and the revision stays
    pf = lib.PreFilter(ctx, lib.PF_DYN4 | lib.PF_FIX4)
    pf.insert(0, ["172.16.0.0/12"])
    batch = [f"{(i >> 8) & 255}.{i & 255}.{(i >> 16) & 255}.0/24" for i in range(65536)]
    with pytest.raises(lib.CvError) as e:
        pf.insert(0, batch)
    assert "Error inserting CIDR string" in str(e.value)
    assert pf.dump() == (["172.16.0.0/12"], 2)
    pf.close()


# ------------------------------------------------------------------ policy map sync
def pkey(ident, dport, proto, egress):
    return struct.pack("<IHBB", ident, ((dport & 0xFF) << 8) | (dport >> 8), proto, egress)


def pval(proxy, packets=0, nbytes=0):
    return struct.pack("<HHHHQQ", ((proxy & 0xFF) << 8) | (proxy >> 8), 0, 0, 0, packets, nbytes)


def map_contents(m):
    k, v = m.dump()
    return {bytes(a): bytes(b) for a, b in zip(k, v)}


def test_policy_sync_desired_realized(ctx):
    m = ctx.map_create(lib.MAP_HASH, 8, 24, 1024)
    s = lib.PolicySync()
    want = {(100, 80, 6, 0): 0, (100, 443, 6, 0): 8080, (7, 0, 0, 1): 0}
    s.set_desired(want)
    assert s.run(ctx, m) == (0, 0, 3, 0)
    assert map_contents(m) == {pkey(*k): pval(p) for k, p in want.items()}      # AllowKey: network order, counters 0
    assert s.realized() == want
    # a datapath hit on an entry the sync leaves alone keeps its counters
    m.update(pkey(100, 80, 6, 0), pval(0, packets=5, nbytes=320))
    # a stale key the agent never wrote is deleted; a changed proxy port is rewritten
    m.update(pkey(9, 53, 17, 0), pval(0))
    want2 = {(100, 80, 6, 0): 0, (100, 443, 6, 0): 9090}
    s.set_desired(want2)
    assert s.run(ctx, m) == (0, 2, 1, 0)                          # deleted (7,..) and (9,..), rewrote 443
    assert map_contents(m) == {pkey(100, 80, 6, 0): pval(0, 5, 320), pkey(100, 443, 6, 0): pval(9090)}
    assert s.realized() == want2
    s.close()


def test_policy_sync_trusts_realized_state(ctx):
    # pkg/endpoint/endpoint.go:2585-2597: only keys whose realized entry is missing or
    # differs are written, so a key the map lost behind the agent's back stays lost
    # while the realized state still holds it
    m = ctx.map_create(lib.MAP_HASH, 8, 24, 64)
    s = lib.PolicySync()
    s.set_desired({(1, 80, 6, 0): 0})
    assert s.run(ctx, m)[2] == 1
    m.delete(pkey(1, 80, 6, 0))
    assert s.run(ctx, m) == (0, 0, 0, 0)
    assert len(m) == 0
    s.close()


def test_policy_sync_counts_failures(ctx):
    m = ctx.map_create(lib.MAP_HASH, 8, 24, 2)                    # room for two keys
    s = lib.PolicySync()
    s.set_desired({(i, 80, 6, 0): 0 for i in range(3)})
    rc, d, a, f = s.run(ctx, m)
    assert rc == -5 and a == 2 and f == 1                         # -EIO: one AllowKey failed (E2BIG)
    assert len(s.realized()) == 2
    s.close()


# ------------------------------------------------------------------ GPU: the agent drives the datapath
def cidr_strings(spec):
    """the distinct CIDRs of a synthetic CIDR map (its key list may repeat a prefix;
    the map holds it once)"""
    out = []
    for k in spec.keys:
        plen = int(struct.unpack("<I", bytes(k[:4]))[0])
        out.append(f"{ipaddress.IPv4Address(bytes(k[4:8]))}/{plen}")
    return list(dict.fromkeys(out))


def cidr_strings_all(spec):
    return [f"{ipaddress.IPv4Address(bytes(k[4:8]))}/{int(struct.unpack('<I', bytes(k[:4]))[0])}" for k in spec.keys]


@pytest.mark.gpu
def test_prefilter_agent_drives_xdp():
    import torch
    assert torch.cuda.is_available()
    w = synth.config1(1 << 16)
    fix, dyn = cidr_strings(w.maps["v4_fix"]), cidr_strings(w.maps["v4_dyn"])
    wp = copy.copy(w)
    wp.maps = {k: v for k, v in w.maps.items() if k not in ("v4_fix", "v4_dyn")}
    ctx, _ = H.product_ctx(wp)
    pf = lib.PreFilter(ctx, lib.PF_DYN4 | lib.PF_FIX4)
    pf.insert(1, fix + dyn)
    dp, _ = H.oracle_dp(w)
    f, l, _ = H.to_dev(w, "cuda:0")
    out = H.dev_out(w.n, "cuda:0")
    ctx.xdp_prefilter(f, l, out)
    o = H.host_out(out)
    assert (o["xdp"] == dp.xdp_prefilter(w.frames, w.length).xdp).all()
    # delete half of each set at revision 2; the next batch sees the smaller sets
    pf.delete(2, fix[::2] + dyn[::2])
    w2 = copy.copy(w)
    w2.maps = dict(w.maps)
    for name, kept in (("v4_fix", set(fix[1::2])), ("v4_dyn", set(dyn[1::2]))):
        sp = copy.copy(w.maps[name])
        rows = [j for j, c in enumerate(cidr_strings_all(w.maps[name])) if c in kept]
        sp.keys, sp.vals = w.maps[name].keys[rows], w.maps[name].vals[rows]
        w2.maps[name] = sp
    dp2, _ = H.oracle_dp(w2)
    out = H.dev_out(w.n, "cuda:0")
    ctx.xdp_prefilter(f, l, out)
    o2 = H.host_out(out)
    ref2 = dp2.xdp_prefilter(w.frames, w.length).xdp
    assert (o2["xdp"] == ref2).all()
    assert (ref2 != dp.xdp_prefilter(w.frames, w.length).xdp).any()
    assert pf.dump()[1] == 3
    pf.close()
    ctx.close()
