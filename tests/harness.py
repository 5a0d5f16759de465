"""Builds the oracle (checker) and the product (HIP library) from one synthetic
workload so parity tests compare them on identical bytes."""
from __future__ import annotations

import numpy as np

from cilium_amd import synth

ROLE_NAMES = ("v4_fix", "v4_dyn", "v6_fix", "v6_dyn", "lxc", "ipcache", "lb4_services", "lb6_services",
              "lb4_revnat", "lb6_revnat")
DEFAULT_MAC = bytes([0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF])          # bpf/lxc_config.h:23 LXC_MAC
NODE_MAC = bytes([0xDE, 0xAD, 0xBE, 0xEF, 0xC0, 0xDE])             # bpf/node_config.h:51


def _ep_cfg(e):
    return dict(ipv4=e.get("ip", 0), ipv6=e.get("ip6", bytes(16)), mac=e.get("mac", DEFAULT_MAC),
                node_mac=e.get("node_mac", NODE_MAC))


def oracle_dp(w: synth.Workload, flags=None, with_ct=True, ct_per_ep=None, ct6_per_ep=None):
    """ct_per_ep: a CT4 MapSpec per endpoint (synth.per_endpoint_ct, ConntrackLocal) instead
    of the global map; maps["ct4_ep"] holds them (ct6_per_ep, maps["ct6_ep"]: the same for CT6)"""
    from oracle import oracle as O
    dp = O.ODp(O.F_DEFAULT if flags is None else flags)
    maps = {}
    for name, spec in w.maps.items():
        if (ct_per_ep is not None and name == "ct4") or (ct6_per_ep is not None and name == "ct6"):
            continue
        maps[name] = O.OMap.from_spec(spec)
        if name in ROLE_NAMES:
            dp.bind(name, maps[name])
    pol = maps.get("policy")
    ct = maps.get("ct4") if with_ct else None
    ct6 = maps.get("ct6") if with_ct else None
    if ct_per_ep is not None:
        maps["ct4_ep"] = [O.OMap.from_spec(s) for s in ct_per_ep]
    if ct6_per_ep is not None:
        maps["ct6_ep"] = [O.OMap.from_spec(s) for s in ct6_per_ep]
    if w.endpoints:
        for k, e in enumerate(w.endpoints):
            i = dp.add_endpoint(e["lxc_id"], e["seclabel"], pol, ct if ct_per_ep is None else maps["ct4_ep"][k])
            dp.endpoint_config(i, ct6=ct6 if ct6_per_ep is None else maps["ct6_ep"][k], **_ep_cfg(e))
    if w.extra and "node" in w.extra:
        dp.node_config(**w.extra["node"])
    dp.keep += [m for k, m in maps.items() if k not in ("ct4_ep", "ct6_ep")] + maps.get("ct4_ep", []) + \
        maps.get("ct6_ep", [])
    return dp, maps


def product_ctx(w: synth.Workload, device=0, flags=None, with_ct=True, ct_per_ep=None, ct6_per_ep=None):
    from cilium_amd import lib
    ctx = lib.Ctx(device, lib.F_DEFAULT if flags is None else flags)
    maps = {}
    for name, spec in w.maps.items():
        if (ct_per_ep is not None and name == "ct4") or (ct6_per_ep is not None and name == "ct6"):
            continue
        maps[name] = ctx.map_from_spec(spec)
        if name in ROLE_NAMES:
            ctx.bind(name, maps[name])
    pol = maps.get("policy")
    ct = maps.get("ct4") if with_ct else None
    ct6 = maps.get("ct6") if with_ct else None
    if ct_per_ep is not None:
        maps["ct4_ep"] = [ctx.map_from_spec(s) for s in ct_per_ep]
    if ct6_per_ep is not None:
        maps["ct6_ep"] = [ctx.map_from_spec(s) for s in ct6_per_ep]
    for k, e in enumerate(w.endpoints):
        i = ctx.endpoint_add(e["lxc_id"], e["seclabel"], pol, ct if ct_per_ep is None else maps["ct4_ep"][k])
        ctx.endpoint_config(i, ct6=ct6 if ct6_per_ep is None else maps["ct6_ep"][k], **_ep_cfg(e))
    if w.extra and "node" in w.extra:
        ctx.node_config(**w.extra["node"])
    ctx.sync()
    return ctx, maps


def to_dev(w: synth.Workload, device="cuda:0", lo=0, hi=None):
    import torch
    hi = w.n if hi is None else hi
    frames = torch.from_numpy(np.ascontiguousarray(w.frames[lo:hi])).to(device)
    length = torch.from_numpy(np.ascontiguousarray(w.length[lo:hi])).to(device)
    mark = torch.from_numpy(np.ascontiguousarray(w.mark[lo:hi])).to(device)
    return frames, length, mark


def egress_inputs(w: synth.Workload, device="cuda:0", lo=0, hi=None):
    """src_ep (int16 view of the u16 endpoint indexes) and flow_hash (int32 view) on the device."""
    import torch
    hi = w.n if hi is None else hi
    src = torch.from_numpy(np.ascontiguousarray(w.extra["src_ep"][lo:hi]).view(np.int16)).to(device)
    fh = torch.from_numpy(np.ascontiguousarray(w.extra["flow_hash"][lo:hi]).view(np.int32)).to(device)
    return src, fh


def dev_out(n, device="cuda:0"):
    import torch
    return {
        "xdp": torch.zeros(n, dtype=torch.uint8, device=device),
        "ret": torch.zeros(n, dtype=torch.int32, device=device),
        "identity": torch.zeros(n, dtype=torch.int32, device=device),
        "ct": torch.zeros(n, dtype=torch.uint8, device=device),
        "proxy": torch.zeros(n, dtype=torch.int16, device=device),
        "nl": torch.zeros(n, dtype=torch.uint8, device=device),
        "nu": torch.zeros(n, dtype=torch.uint8, device=device),
        "reason": torch.zeros(n, dtype=torch.int32, device=device),
    }


def host_out(out):
    import torch
    torch.cuda.synchronize()
    r = {k: v.cpu().numpy() for k, v in out.items()}
    r["identity"] = r["identity"].view(np.uint32)
    r["proxy"] = r["proxy"].view(np.uint16)
    return r


def sorted_rows(keys, vals):
    rows = np.concatenate([keys, vals], axis=1)
    order = np.lexsort(keys.T[::-1])
    return rows[order]


def rows_diff(a, b):
    """where two sorted_rows tables differ: the row count, or the differing byte columns
    and the first differing row of each (for assertion messages)"""
    if a.shape != b.shape:
        return f"shapes {a.shape} vs {b.shape}"
    bad = np.nonzero((a != b).any(axis=0))[0]
    r = np.nonzero((a != b).any(axis=1))[0]
    return f"{len(r)} rows differ in byte columns {bad.tolist()}; first: {a[r[0]].tolist()} vs {b[r[0]].tolist()}" \
        if len(r) else "equal"


def apply_variant(frames, rows, offs, ports):
    """frames with the 2-byte big-endian ports of synth.port_variant written in"""
    out = frames.copy()
    out[rows, offs] = (ports >> 8).astype(np.uint8)
    out[rows, offs + 1] = (ports & 0xFF).astype(np.uint8)
    return out


class ShardedOracle:
    """The ingress oracle run the way the GPU runs it: packets partitioned by
    direction-symmetric address pair (cilium_amd.shard, the config-4 key), one
    datapath per shard holding that shard's conntrack entries, shards processed on
    parallel host threads (ctypes releases the GIL).  Address pairs share no CT
    entry, so the union equals one sequential run (tests/test_multi_rank.py)."""

    def __init__(self, w: synth.Workload, threads: int):
        from concurrent.futures import ThreadPoolExecutor
        from cilium_amd import shard
        self.T = max(1, threads)
        self.w = w
        split = shard.split_workload_all(w, self.T)
        with ThreadPoolExecutor(self.T) as ex:                     # (the C loads release the GIL)
            dps = list(ex.map(lambda po: oracle_dp(po[0]), split))
        self.parts = [(own, dp, maps) for (_, own), (dp, maps) in zip(split, dps)]

    def netdev_ingress(self, frames=None, now=None, pool=None):
        """verdicts of the whole batch (packet order) and the parallel section's wall time"""
        import time
        from concurrent.futures import ThreadPoolExecutor
        w = self.w
        frames = w.frames if frames is None else frames
        now = w.now if now is None else now
        inputs = [(np.ascontiguousarray(frames[own]), np.ascontiguousarray(w.length[own]),
                   np.ascontiguousarray(w.mark[own])) for own, _, _ in self.parts]
        run = lambda t: self.parts[t][1].netdev_ingress(*inputs[t], now=now)
        ex = pool or ThreadPoolExecutor(self.T)
        t0 = time.perf_counter()
        outs = list(ex.map(run, range(self.T)))
        el = time.perf_counter() - t0
        if pool is None:
            ex.shutdown()
        from oracle import oracle as O
        res = O.Out(w.n)
        for (own, _, _), o in zip(self.parts, outs):
            for k in O.Out.FIELDS:
                getattr(res, k)[own] = getattr(o, k)
        return res, el

    def metrics(self):
        return sum(dp.metrics() for _, dp, _ in self.parts)

    def dump(self, name):
        ks, vs = zip(*(maps[name].dump() for _, _, maps in self.parts))
        return np.concatenate(ks), np.concatenate(vs)

    def digest(self, name):
        """table_digest of the union of the shards' tables (disjoint key sets)"""
        cnt, tot, x = 0, 0, 0
        for _, _, maps in self.parts:
            c, s, y = maps[name].digest()
            cnt, tot, x = cnt + c, (tot + s) & 0xFFFFFFFFFFFFFFFF, x ^ y
        return (cnt, tot, x)

    def policy_rows(self, name="policy"):
        """the policy map as one node's: every shard's packets / bytes counters summed
        (the agent sums per-rank counters), key-sorted rows"""
        base = None
        tot = None
        for _, _, maps in self.parts:
            rows = sorted_rows(*maps[name].dump())
            if base is None:
                base = rows.copy()
                tot = np.zeros((len(rows), 2), np.uint64)
            assert (rows[:, :16] == base[:, :16]).all()
            tot += rows[:, 16:32].copy().view("<u8").reshape(-1, 2)
        spec = self.w.maps[name]
        init = sorted_rows(spec.keys, spec.vals)[:, 16:32].copy().view("<u8").reshape(-1, 2)
        with np.errstate(over="ignore"):
            tot -= init * np.uint64(len(self.parts) - 1)
        base[:, 16:32] = tot.view(np.uint8).reshape(-1, 16)
        return base


class FamilyOracle:
    """Config 5's oracle the way bench.py runs the GPU: the IPv4 packets and the IPv6
    packets as two batches (64-B and 128-B records).  Their conntrack, service and
    reverse-NAT state is disjoint (CT4 / lb4 vs CT6 / lb6; LXC_NAT46 off); they share only
    additive state -- the policy counters and cilium_metrics -- so one datapath per family
    on its own host thread, counters summed, equals one sequential run."""

    def __init__(self, w):
        from concurrent.futures import ThreadPoolExecutor
        self.w = w
        with ThreadPoolExecutor(2) as ex:
            self.dps = list(ex.map(lambda _: oracle_dp(w), range(2)))

    def lxc_egress(self, parts, frames, now):
        """per family: the oracle's outputs for its part of the step's frames"""
        from concurrent.futures import ThreadPoolExecutor
        run = lambda k: self.dps[k][0].lxc_egress(frames[k], parts[k]["length"], parts[k]["src_ep"],
                                                  parts[k]["flow_hash"], now=now)
        with ThreadPoolExecutor(2) as ex:
            return list(ex.map(run, range(2)))

    def metrics(self):
        return sum(dp.metrics() for dp, _ in self.dps)

    def policy_rows(self):
        rows = [sorted_rows(*maps["policy"].dump()) for _, maps in self.dps]
        assert (rows[0][:, :16] == rows[1][:, :16]).all()
        init = sorted_rows(self.w.maps["policy"].keys, self.w.maps["policy"].vals)[:, 16:32].copy().view("<u8")
        c = [r[:, 16:32].copy().view("<u8") for r in rows]
        out = rows[0].copy()
        with np.errstate(over="ignore"):
            out[:, 16:32] = (c[0] + c[1] - init).view(np.uint8)
        return out

    def digest(self, name):
        return self.dps[0 if name == "ct4" else 1][1][name].digest()


def _dg_mix(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def table_digest(keys, vals, chunk=1 << 22):
    """(count, sum, xor) of the entries' chains, the same function as the oracle's
    or_map_digest: key then value, each zero-padded to 8-byte words, chained through
    splitmix64's finalizer.  Order-independent: compares a full-size table dump with
    the oracle's without sorting 33M rows."""
    n = len(keys)
    tot, x = np.uint64(0), np.uint64(0)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        h = np.full(hi - lo, 0x243F6A8885A308D3, np.uint64)
        for part in (keys[lo:hi], vals[lo:hi]):
            w = part.shape[1]
            pad = np.zeros((hi - lo, (w + 7) // 8 * 8), np.uint8)
            pad[:, :w] = part
            words = pad.view("<u8")
            for j in range(words.shape[1]):
                h = _dg_mix(h ^ words[:, j])
        with np.errstate(over="ignore"):
            tot = tot + np.add.reduce(h, dtype=np.uint64)
        x ^= np.bitwise_xor.reduce(h)
    return (n, int(tot), int(x))

