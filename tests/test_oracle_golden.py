"""The CPU oracle pinned against the reference and the kernel.

* test/bpf/unit-test.c known answers (GET_PREFIX / LPM_LOOKUP_FN prefixes,
  ipv6_addr_clear_suffix), plus an exhaustive comparison with the reference's own
  helpers compiled from /root/reference into oracle/_ref (when built);
* struct layouts vs the reference headers (oracle/_ref probe);
* kernel map semantics (update/delete/lookup return codes and results);
* config 1 XDP verdicts vs BPF_PROG_TEST_RUN of the bpf_xdp.c restatement;
* config 2 ingress verdicts, identities and policy counters vs BPF_PROG_TEST_RUN.
"""
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O


def load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


def ntohl(x):
    return struct.unpack(">I", struct.pack("<I", x))[0]


def test_get_prefix_unit_test_kats():
    # test/bpf/unit-test.c:59-102: match_dummy_prefix(addr & GET_PREFIX(p)) == stored
    L = O.lib()
    gp = lambda p: L.or_get_prefix(p)
    def match(addr_be, stored_be, p):
        return (addr_be & gp(p)) == stored_be
    h = lambda x: ntohl(x)  # htonl on LE
    assert match(h(0xFFFFFFFF), h(0xFFFFFFFF), 32)
    assert not match(h(0xFFF00000), h(0xFFFFFFFF), 32)
    assert match(h(0xFFFFFFFE), h(0xFFFFFFFE), 31)
    assert match(h(0xFFFFFFFF), h(0xFFFFFFFE), 31)
    assert not match(h(0xFFF00000), h(0xFFFFFFFE), 31)
    assert match(h(0xFFFFFC00), h(0xFFFFFC00), 22)
    assert match(h(0xFFFFFFFF), h(0xFFFFFC00), 22)
    assert not match(h(0xFFF00000), h(0xFFFFFC00), 22)
    assert match(h(0xFFE00000), h(0xFFE00000), 11)
    assert match(h(0xFFFFFFFF), h(0xFFE00000), 11)
    assert match(h(0xFFF00000), h(0xFFE00000), 11)
    assert match(h(0xF0000000), h(0xF0000000), 11)
    assert match(h(0x00000000), h(0x00000000), 0)
    assert match(h(0xFFFFFFFF), h(0x00000000), 0)


def test_clear_suffix_unit_test_kats():
    # test/bpf/unit-test.c:20-57
    L = O.lib()
    for prefix, words in [(128, [0xffffffff] * 4), (127, [0xffffffff] * 3 + [0xfffffffe]),
                          (95, [0xffffffff, 0xffffffff, 0xfffffffe, 0]), (1, [0x80000000, 0, 0, 0]),
                          (-1, [0, 0, 0, 0])]:
        a = np.full(16, 0xFF, np.uint8)
        L.or_ipv6_addr_clear_suffix(a.ctypes.data, prefix)
        got = [int.from_bytes(a[4 * i:4 * i + 4].tobytes(), "big") for i in range(4)]
        assert got == words, prefix


def test_helpers_vs_reference_build():
    R = O.ref_probe()
    if R is None:
        pytest.skip("oracle/_ref not built (reference tree absent)")
    L = O.lib()
    for p in range(-40, 170):
        assert L.or_get_prefix(p) == R.ref_get_prefix(p), p
    rng = np.random.default_rng(1)
    for p in range(-5, 140):
        for _ in range(8):
            a = rng.integers(0, 256, 16, dtype=np.uint8)
            b = a.copy()
            L.or_ipv6_addr_clear_suffix(a.ctypes.data, p)
            R.ref_ipv6_addr_clear_suffix(b.ctypes.data, p)
            assert (a == b).all(), p


def test_struct_layouts_vs_reference_build():
    R = O.ref_probe()
    if R is None:
        pytest.skip("oracle/_ref not built")
    n = R.ref_layout(-1)
    got = [R.ref_layout(i) for i in range(n)]
    # sizes: lpm_v4_key lpm_v6_key lpm_val endpoint_key endpoint_info ipcache_key
    # remote_endpoint_info policy_key policy_entry metrics_key metrics_value
    # ipv4_ct_tuple ipv6_ct_tuple ct_entry lb4_key lb4_service lb6_key lb6_service
    sizes = [8, 20, 1, 20, 48, 24, 8, 8, 24, 8, 16, 14, 40, 56, 8, 12, 20, 24]
    offs = [16, 6, 8, 7, 8, 8, 8, 12, 32, 38, 40, 42, 43, 44, 48, 52, 32, 36]
    assert got == sizes + offs


def test_map_semantics_vs_kernel(golden_dir):
    g = load(golden_dir, "map_semantics_kernel.npz")
    for c in range(int(g["ncases"])):
        typ, ks, vs, mx = (int(x) for x in g[f"c{c}_meta"])
        m = O.OMap(typ, ks, vs, mx)
        for i, op in enumerate(g[f"c{c}_op"]):
            k, v = g[f"c{c}_key"][i].tobytes(), g[f"c{c}_val"][i].tobytes()
            fl, rc = int(g[f"c{c}_flags"][i]), int(g[f"c{c}_rc"][i])
            if op == 0:
                assert m.update(k, v, fl) == rc, (c, i)
            elif op == 1:
                assert m.delete(k) == rc, (c, i)
            else:
                r, val = m.lookup(k)
                assert r == rc, (c, i)
                if r == 0:
                    assert val == v, (c, i)


def _maps_from(g, prefix="map_"):
    maps = {}
    for key in g:
        if key.startswith(prefix) and key.endswith("_meta"):
            name = key[len(prefix):-5]
            t, ks, vs, mx = (int(x) for x in g[key])
            m = O.OMap(t, ks, vs, mx)
            m.load(g[f"{prefix}{name}_keys"], g[f"{prefix}{name}_vals"])
            maps[name] = m
    return maps


def test_config1_xdp_vs_kernel(golden_dir):
    g = load(golden_dir, "c1_xdp_kernel.npz")
    dp = O.ODp()
    for name, m in _maps_from(g).items():
        dp.bind(name, m)
    out = dp.xdp_prefilter(g["frames"], g["length"])
    assert (out.xdp == g["verdict"]).all()
    assert set(np.unique(out.xdp)) == {1, 2}


def test_config2_policy_vs_kernel(golden_dir):
    g = load(golden_dir, "c2_policy_kernel.npz")
    maps = _maps_from(g)
    dp = O.ODp()
    dp.bind("ipcache", maps["ipcache"])
    dp.add_endpoint(1, 0x1010, maps["policy"])
    out = dp.policy_ingress(0, g["frames"], g["length"], g["mark"])
    assert (out.ret == g["ret"]).all()
    assert (out.identity == g["identity"]).all()
    # policy counters after the run, per key, vs the kernel map
    pol = maps["policy"]
    for i, k in enumerate(g["map_policy_keys"]):
        r, v = pol.lookup(k.tobytes())
        assert r == 0 and v == g["policy_vals_after"][i].tobytes(), i
    # drops land in cilium_metrics (reason = -ret, dir ingress)
    met = dp.metrics()
    for code in np.unique(g["ret"][g["ret"] < 0]):
        cnt = int((g["ret"] == code).sum())
        assert int(met[-code, 1, 0]) == cnt


def test_checksum_helpers_vs_kernel(golden_dir):
    """bpf_l3_csum_replace / bpf_l4_csum_replace / bpf_csum_diff as the container's
    kernel computes them (BPF_PROG_TEST_RUN, oracle/kernel_golden.py gen_csum): the
    arithmetic of every packet rewrite (lb4_xlate, __lb4_rev_nat, ipv4_dec_ttl)."""
    import struct
    from oracle.oracle import csum_apply
    g = np.load(os.path.join(golden_dir, "csum_kernel.npz"))
    fin, fout = g["frames_in"], g["frames_out"]
    n = {0: 0, 1: 0, 2: 0}
    for i in range(len(fin)):
        op, off, frm, to, flags = struct.unpack("<IIIII", fin[i, 64:84].tobytes())
        rc, after, diff = csum_apply(fin[i].tobytes(), op, off, frm, to, flags)
        assert rc == 0, i
        if op == 2:
            assert diff == struct.unpack("<Q", fout[i, 84:92].tobytes())[0], i
        else:
            assert after[off:off + 2] == fout[i, off:off + 2].tobytes(), (i, op, flags)
        n[op] += 1
    assert min(n.values()) > 1000


def test_csum_diff16_vs_kernel(golden_dir):
    """bpf_csum_diff over two 16-byte IPv6 addresses as the container's kernel computes
    it (oracle/kernel_golden.py gen_csum16): the sum of lb6_xlate and __lb6_rev_nat."""
    import struct
    from oracle.oracle import csum_apply
    g = np.load(os.path.join(golden_dir, "csum16_kernel.npz"))
    fin, fout = g["frames_in"], g["frames_out"]
    for i in range(len(fin)):
        seed = struct.unpack("<I", fin[i, 96:100].tobytes())[0]
        rc, _, diff = csum_apply(fin[i, 64:96].tobytes(), 3, 0, 0, 0, seed)
        assert rc == 0
        assert diff == struct.unpack("<Q", fout[i, 104:112].tobytes())[0], (i, fin[i, 64:100].tobytes().hex())
    assert len(fin) >= 4000
