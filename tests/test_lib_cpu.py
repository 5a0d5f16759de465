"""CPU-side checks of the product library: it builds, loads, exports every symbol
include/cilium_hip.h declares, and its map store (host-only context) reproduces the
kernel's map semantics on the golden sequences (no GPU compute is invoked)."""
import os
import subprocess

import numpy as np
import pytest

from cilium_amd import lib, synth


def test_library_exports_header_symbols():
    L = lib.load()
    names = lib.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}" in out, n


def test_library_is_gfx950_code_object():
    out = subprocess.run(["strings", lib.LIB_PATH], capture_output=True, text=True)
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in out.stdout


def test_host_only_ctx_rejects_batches():
    ctx = lib.Ctx(-1)
    m = ctx.map_create(lib.MAP_HASH, 8, 24, 16)
    assert m.update(b"\1" * 8, b"\2" * 24) == 0
    import ctypes as C
    b = lib.Batch(None, 64, None, None, 0)
    o = lib.Out()
    assert lib.load().cv_xdp_prefilter(ctx.h, C.byref(b), C.byref(o), None) == -19   # -ENODEV


def test_map_semantics_vs_kernel(golden_dir):
    g = np.load(os.path.join(golden_dir, "map_semantics_kernel.npz"))
    ctx = lib.Ctx(-1)
    for c in range(int(g["ncases"])):
        typ, ks, vs, mx = (int(x) for x in g[f"c{c}_meta"])
        m = ctx.map_create(typ, ks, vs, mx)
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


def test_get_next_key_walks_every_element():
    ctx = lib.Ctx(-1)
    m = ctx.map_create(lib.MAP_HASH, 8, 4, 1000)
    keys = {np.random.default_rng(3).integers(0, 2**63).item().to_bytes(8, "little") for _ in range(300)}
    for k in keys:
        assert m.update(k, b"\0" * 4) == 0
    seen, k = set(), None
    while True:
        rc, nk = m.next_key(k)
        if rc:
            break
        seen.add(nk)
        k = nk
    assert seen == keys
    # absent key -> first element (kernel hashtab semantics)
    rc, first = m.next_key(b"\xff" * 8)
    assert rc == 0 and first in keys


def test_bind_checks_layouts():
    ctx = lib.Ctx(-1)
    bad = ctx.map_create(lib.MAP_HASH, 8, 1, 10)
    with pytest.raises(lib.CvError):
        ctx.bind("v4_dyn", bad)          # v4_dyn must be an LPM_TRIE
    with pytest.raises(lib.CvError):
        ctx.bind("lxc", bad)
    ok = ctx.map_create(lib.MAP_LPM_TRIE, 24, 8, 10)
    ctx.bind("ipcache", ok)


def test_ct_gc_host_store_vs_oracle():
    """ctmap.GC(GCFilterByTime) on an unbound CT map (host store) against the oracle's
    restatement of doFiltering (pkg/maps/ctmap/ctmap.go:401-410), then Flush."""
    from cilium_amd import synth
    from oracle.oracle import OMap
    w = synth.config3(256, 4096, n_ep=8, n_cidrs=256, n_ids=20, seed=5)
    spec = w.maps["ct4"]
    life = np.ascontiguousarray(spec.vals[:, 32:36]).view("<u4").ravel()
    vals = spec.vals.copy()                       # spread the lifetimes: every third entry older
    vals[::3, 32:36] = (life[::3] - 5000).astype("<u4").view(np.uint8).reshape(-1, 4)
    life = np.ascontiguousarray(vals[:, 32:36]).view("<u4").ravel()
    t = int(np.median(life))
    ctx = lib.Ctx(-1)
    m = ctx.map_create(spec.type, spec.key_size, spec.val_size, spec.max_entries)
    m.update_batch(spec.keys, vals)
    om = OMap(spec.type, spec.key_size, spec.val_size, spec.max_entries)
    om.load(spec.keys, vals)
    _, ov = om.dump()                             # (the spec repeats shared RELATED twins)
    live = np.ascontiguousarray(ov[:, 32:36]).view("<u4").ravel()
    want = int((live < t).sum())
    assert 0 < want < len(live) == len(m)
    assert m.ct_gc(t) == om.ct_gc(t) == want
    assert len(m) == len(om) == len(live) - want
    k1, v1 = m.dump()
    k2, v2 = om.dump()
    rows = lambda k, v: sorted(bytes(a) + bytes(b) for a, b in zip(k, v))
    assert rows(k1, v1) == rows(k2, v2)
    assert m.ct_gc(t) == 0                        # idempotent
    assert m.ct_gc(0xFFFFFFFF) == om.ct_gc(0xFFFFFFFF) == len(live) - want   # ctmap.Flush
    assert len(m) == 0


def test_concurrent_agent_writers():
    """SURVEY.md §8(b) threading: agent goroutines update maps concurrently (the C-ABI
    serialises per context).  8 threads insert, overwrite and delete disjoint key
    ranges of one hash map and one LPM map at once; the final contents are exactly the
    union of what each thread left, and the counts agree."""
    import threading
    ctx = lib.Ctx(-1)
    hm = ctx.map_create(lib.MAP_HASH, 8, 24, 1 << 16)
    lm = ctx.map_create(lib.MAP_LPM_TRIE, 24, 8, 1 << 16, lib.BPF_F_NO_PREALLOC)
    T, N = 8, 1500
    errs = []

    def key8(t, i):
        return np.array([t * 100000 + i, 6 << 16 | 80], np.uint32).tobytes()

    def key24(t, i):
        return synth.ipcache_keys_v4(np.array([(10 << 24) | (t << 16) | (i << 4)], np.uint32),
                                     np.array([28]))[0].tobytes()

    def worker(t):
        try:
            for i in range(N):
                assert hm.update(key8(t, i), bytes([t]) * 24) == 0
                assert lm.update(key24(t, i), np.array([t, i], np.uint32).tobytes()) == 0
            for i in range(0, N, 3):
                assert hm.delete(key8(t, i)) == 0
                assert lm.delete(key24(t, i)) == 0
            for i in range(1, N, 3):
                assert hm.update(key8(t, i), bytes([t + 100]) * 24, 2) == 0   # BPF_EXIST
        except AssertionError as e:  # noqa: PERF203
            errs.append((t, repr(e)))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:3]
    keep = [i for i in range(N) if i % 3]
    assert len(hm) == T * len(keep) and len(lm) == T * len(keep)
    for t in range(T):
        for i in range(N):
            rc, v = hm.lookup(key8(t, i))
            if i % 3 == 0:
                assert rc == -2
            else:
                assert rc == 0 and v == bytes([t + 100 if i % 3 == 1 else t]) * 24
            rc, v = lm.lookup(key24(t, i))
            assert (rc == -2) if i % 3 == 0 else (rc == 0 and v == np.array([t, i], np.uint32).tobytes())
