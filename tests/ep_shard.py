"""Config 5 across ranks as ONE node, with endpoint-owned conntrack -- a CPU prototype
(TEST INFRASTRUCTURE: the oracle is the datapath of every rank here).

The reference can give every endpoint its own CT maps (CT_MAP4 / CT_MAP6 are per-program
macros, bpf_lxc.c:53-75; per-endpoint map names when the endpoint's conntrack is local).
Rank r owns the endpoints e with e % world == r and their maps.  A packet's source
program -- handle_ipv4_from_lxc / ipv6_l3_from_lxc: the service lookup and lb4_local /
lb6_local on the source's map, the egress ct_lookup / ct_create, the egress policy --
runs on its source's rank; its local delivery -- the destination's ipv4_policy /
ipv6_policy on the destination's map -- runs on the destination's rank, from the frame
the source program left (oracle or_lxc_egress_split / or_lxc_deliver).

Exact by construction: a CT map is touched only by its endpoint's source programs and by
deliveries into it, and an entry of it is keyed by the endpoint's address and a peer
address, so every rank applies the operations of a map that share a peer in packet
order; policy counters and metrics are sums.  An operation waits only for earlier ones
of its map that share a peer and have not run -- in the end, for a delivery whose source
program (on another rank) has not run yet.  Candidate destinations and peers come from
the headers and the read-only tables (candidates: the destination address's endpoint,
or a VIP's local backends; peers: see `peers`), as supersets; a source program that
delivers anywhere else fails the run loudly.  A round is local progress until every
map waits, then one exchange (all_gather of the delivery records and of the "not for
you" resolutions of the other candidates).  Rounds grow with the longest chain of
cross-rank request / reply alternations within one address pair, not with the batch.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Sequence

import numpy as np

from cilium_amd import synth

DEFER = -3                      # OR_E_DEFER
# the most CT entries one operation creates in its map: a source program its service entry,
# the tuple, its ICMP twin and the NAT tuple (lb4_local, ct_create4: lb.h:700-775,
# conntrack.h:663-744) -- 7 bounds it as cv_lxc_egress does; a delivery the tuple and its twin
MAX_CREATES = (7, 2)


def per_endpoint_dp(w: synth.Workload):
    """An oracle datapath of w whose endpoints each own a fresh CT4 and CT6 map."""
    from oracle import oracle as O
    from tests import harness as H
    dp = O.ODp(O.F_DEFAULT)
    maps = {}
    for name, spec in w.maps.items():
        if name in ("ct4", "ct6"):
            continue
        maps[name] = O.OMap.from_spec(spec)
        if name in H.ROLE_NAMES:
            dp.bind(name, maps[name])
    c4, c6 = w.maps["ct4"], w.maps["ct6"]
    maps["ct4"], maps["ct6"] = [], []
    for e in w.endpoints:
        m4 = O.OMap(c4.type, c4.key_size, c4.val_size, c4.max_entries)
        m6 = O.OMap(c6.type, c6.key_size, c6.val_size, c6.max_entries)
        i = dp.add_endpoint(e["lxc_id"], e["seclabel"], maps["policy"], m4)
        dp.endpoint_config(i, ct6=m6, **H._ep_cfg(e))
        maps["ct4"].append(m4)
        maps["ct6"].append(m6)
    if w.extra and "node" in w.extra:
        dp.node_config(**w.extra["node"])
    dp.keep += [m for m in maps.values() if not isinstance(m, list)]
    return dp, maps


# the prototype's node tables, candidates and peers (the product's are cv_epnode.cpp's,
# from the context's own tables; test_ep_sched_matches_prototype compares them)
def node_tables(endpoints: Sequence[dict], services: Dict[str, tuple]):
    """address -> local endpoints; VIP -> backend addresses; backend address -> VIPs.
    services: {"lb4_services": (keys, vals), "lb6_services": (keys, vals)} as the agent
    wrote them (lb4_key / lb4_service, lb.h): slave entries (slave != 0) name backends."""
    where, backends, vips = {}, {}, {}
    for idx, e in enumerate(endpoints):
        if e.get("ip"):
            where.setdefault(struct.pack(">I", e["ip"]), set()).add(idx)
        if e.get("ip6") and any(e["ip6"]):
            where.setdefault(bytes(e["ip6"]), set()).add(idx)
    for name, alen in (("lb4_services", 4), ("lb6_services", 16)):
        if name not in services:
            continue
        keys, vals = services[name]
        slave = keys[:, alen + 2] | (keys[:, alen + 3].astype(np.int64) << 8)
        for k, v in zip(keys[slave > 0], vals[slave > 0]):
            vip, be = bytes(k[:alen]), bytes(v[:alen])
            backends.setdefault(vip, set()).add(be)
            vips.setdefault(be, set()).add(vip)
    return where, backends, vips


def _addrs(f):
    """(saddr, daddr) bytes of a frame, or None"""
    if f[12] == 0x08 and f[13] == 0x00:
        return bytes(f[26:30]), bytes(f[30:34])
    if f[12] == 0x86 and f[13] == 0xDD:
        return bytes(f[22:38]), bytes(f[38:54])
    return None


def candidates_of(frames: np.ndarray, tables) -> List[frozenset]:
    """per packet, the endpoints its source program may deliver it to (a superset): the
    destination address's endpoint, or the local backends of the VIP it is"""
    where, backends, _ = tables
    out = []
    for f in frames:
        a = _addrs(f)
        c = set()
        if a is not None:
            c |= where.get(a[1], set())
            for be in backends.get(a[1], ()):
                c |= where.get(be, set())
        out.append(frozenset(c))
    return out


def peers_of(frames: np.ndarray, tables, loopback: int):
    """per packet, the peer addresses of the CT entries its source program (on the
    source's map) and its delivery (on the destination's map) may touch -- supersets.
    The source program's peer is the destination address, or a VIP's backends (its
    service entry, the translated connection, the NAT tuple) and, when the client backs
    the VIP itself, the loopback address; the delivery's is the source address as the
    source program left it: the original, a VIP (reverse NAT of a backend's reply) or the
    loopback address."""
    _, backends, vips = tables
    lob = struct.pack(">I", loopback) if loopback else b""
    src_p, dst_p = [], []
    for f in frames:
        a = _addrs(f)
        if a is None:
            src_p.append(frozenset())
            dst_p.append(frozenset())
            continue
        loop = lob and a[0] in backends.get(a[1], ())                # a VIP the client itself backs
        sp = {a[1]} | backends.get(a[1], set()) | ({lob} if loop else set())
        dp = {a[0]} | vips.get(a[0], set()) | ({lob} if loop else set())
        src_p.append(frozenset(sp))
        dst_p.append(frozenset(dp))
    return src_p, dst_p


def _tables(w: synth.Workload):
    return node_tables(w.endpoints, {k: (w.maps[k].keys, w.maps[k].vals) for k in ("lb4_services", "lb6_services")
                                     if k in w.maps})


def candidates(w: synth.Workload):
    """per packet, the endpoints its source program may deliver it to (a superset)"""
    return candidates_of(w.frames, _tables(w))


def peers(w: synth.Workload):
    """per packet, the peer addresses its source program and its delivery may touch (supersets)"""
    lo = w.extra.get("node", {}).get("loopback", 0) if w.extra else 0
    return peers_of(w.frames, _tables(w), lo)


class RankState:
    """One rank's endpoints, their maps and their operations in packet order."""

    FIELDS = ("ret", "identity", "ct", "proxy", "nl", "nu", "reason")

    def __init__(self, w: synth.Workload, rank: int, world: int, now: int, cand=None, peer_sets=None):
        self.w, self.rank, self.world, self.now = w, rank, world, now
        self.dp, self.maps = per_endpoint_dp(w)
        self.cand = candidates(w) if cand is None else cand
        src_p, dst_p = peers(w) if peer_sets is None else peer_sets
        n_ep = len(w.endpoints)
        self.owned = [e for e in range(n_ep) if e % world == rank]
        src = w.extra["src_ep"]
        ops = {e: [] for e in self.owned}
        for i in range(w.n):
            s = int(src[i])
            if s % world == rank:
                ops[s].append((i, 0, src_p[i]))
            for d in self.cand[i]:
                if d % world == rank:
                    ops[d].append((i, 1, dst_p[i]))
        # (packet, source before delivery): the order the sequential run applies them in
        self.pending = {e: sorted(v, key=lambda o: (o[0], o[1])) for e, v in ops.items()}
        self.resolved = {}                       # (packet, endpoint) -> delivery record or None
        self.v6 = (w.frames[:, 12] == 0x86) & (w.frames[:, 13] == 0xDD)   # (the op's map: CT6, else CT4)
        self.out = {k: np.zeros(w.n, np.int64) for k in self.FIELDS}
        self.mine = np.zeros(w.n, bool)          # outputs final on this rank
        self.cross = 0                           # deliveries whose source ran on another rank

    def _source(self, i, outbox):
        w = self.w
        o, dl, ifx, lab = self.dp.lxc_egress_split(w.frames[i:i + 1], w.length[i:i + 1], w.extra["src_ep"][i:i + 1],
                                                   w.extra["flow_hash"][i:i + 1], now=self.now)
        dst = int(dl[0]) if o.ret[0] == DEFER else -1
        if dst >= 0 and dst not in self.cand[i]:
            raise AssertionError(f"packet {i} delivered to endpoint {dst}, not a candidate {sorted(self.cand[i])}")
        rec = None
        if dst >= 0:
            rec = {"frame": o.frames_out[0].copy(), "ifindex": int(ifx[0]), "label": int(lab[0]),
                   "identity": int(o.identity[0]), "ct": int(o.ct[0]), "nl": int(o.nl[0]), "nu": int(o.nu[0])}
        else:
            for k in self.FIELDS:
                self.out[k][i] = getattr(o, k)[0]
            self.mine[i] = True
        for d in self.cand[i] | ({dst} if dst >= 0 else set()):
            r = rec if d == dst else None
            if d % self.world == self.rank:
                self.resolved[(i, d)] = r
            else:
                outbox.setdefault(d % self.world, []).append((i, d, r))

    def _deliver(self, i, d, rec):
        w = self.w
        o = self.dp.lxc_deliver(rec["frame"][None, :], w.length[i:i + 1], [d], [rec["ifindex"]], [rec["label"]],
                                [rec["nl"]], [rec["nu"]], now=self.now)
        for k in ("ret", "proxy", "nl", "nu", "reason"):
            self.out[k][i] = getattr(o, k)[0]
        self.out["identity"][i] = rec["identity"]
        self.out["ct"][i] = rec["ct"]
        self.mine[i] = True
        if int(self.w.extra["src_ep"][i]) % self.world != self.rank:
            self.cross += 1

    def _tight(self, e):
        """per family, whether endpoint e's CT map may reach max_entries with the creates its
        pending operations may still make (MAX_CREATES per operation kind): then the creates
        of different peers compete for the room, and the map's operations keep packet order
        across all peers (conntrack.h:692-693: a create that finds the map full fails)"""
        v6 = self.v6
        need = [0, 0]
        for i, kind, _ in self.pending[e]:
            need[int(v6[i])] += MAX_CREATES[kind]
        return [len(self.maps[f][e]) + need[k] > self.maps[f][e].max_entries for k, f in enumerate(("ct4", "ct6"))]

    def progress(self):
        """local operations until every owned map waits; returns {rank: records}.  A map's
        operation runs once every earlier operation of that map sharing a peer with it
        has run (a delivery whose source program has not run yet blocks its peers); on a
        map that may fill (`_tight`), once every earlier operation of the map has run."""
        outbox = {}
        moved = True
        while moved:
            moved = False
            for e in self.owned:
                blocked, left = set(), []
                tight, stop = self._tight(e), [False, False]
                for op in self.pending[e]:
                    i, kind, pe = op
                    fam = int(self.v6[i])
                    ready = kind == 0 or (i, e) in self.resolved
                    if not ready or (pe & blocked) or stop[fam]:
                        blocked |= pe
                        stop[fam] |= tight[fam]
                        left.append(op)
                        continue
                    if kind == 0:
                        self._source(i, outbox)
                    else:
                        rec = self.resolved.pop((i, e))
                        if rec is not None:
                            self._deliver(i, e, rec)
                    moved = True
                self.pending[e] = left
        return outbox

    def receive(self, records):
        for i, d, r in records:
            self.resolved[(i, d)] = r

    def done(self):
        return not any(self.pending[e] for e in self.owned)

    def result(self):
        ct = {}
        for e in self.owned:
            ct[e] = (self.maps["ct4"][e].dump(), self.maps["ct6"][e].dump())
        return {"out": {k: v[self.mine] for k, v in self.out.items()}, "idx": np.nonzero(self.mine)[0],
                "ct": ct, "metrics": self.dp.metrics(), "policy": self.maps["policy"].dump(), "cross": self.cross}


def simulate(w: synth.Workload, world: int, now: int):
    """every rank in one process, in lockstep rounds; (results, rounds)"""
    cand, ps = candidates(w), peers(w)
    ranks = [RankState(w, r, world, now, cand, ps) for r in range(world)]
    rounds = 0
    while not all(r.done() for r in ranks):
        boxes = [r.progress() for r in ranks]
        rounds += 1
        for b in boxes:
            for dest, recs in b.items():
                ranks[dest].receive(recs)
        if rounds > w.n + 2:
            raise AssertionError("no progress")
    return [r.result() for r in ranks], rounds


def merge(w: synth.Workload, results):
    """the ranks' results as one node's: outputs, per-endpoint tables, metrics, policy
    counters (each rank adds its deltas to the shared initial values)"""
    out = {k: np.zeros(w.n, np.int64) for k in RankState.FIELDS}
    seen = np.zeros(w.n, int)
    ct = {}
    metrics = np.zeros((256, 4, 2), np.uint64)
    init_k, init_v = w.maps["policy"].keys, w.maps["policy"].vals
    pol = None
    for r in results:
        for k in RankState.FIELDS:
            out[k][r["idx"]] = r["out"][k]
        seen[r["idx"]] += 1
        ct.update(r["ct"])
        metrics += r["metrics"]
        pk, pv = r["policy"]
        order = np.lexsort(pk.T[::-1])
        pk, pv = pk[order], pv[order].copy()
        if pol is None:
            io = np.lexsort(init_k.T[::-1])
            base = init_v[io].copy()
            pol = [pk, base.copy(), base]
        cnt = pv[:, 8:24].copy().view("<u8") - pol[2][:, 8:24].copy().view("<u8")
        acc = pol[1][:, 8:24].copy().view("<u8") + cnt
        pol[1][:, 8:24] = acc.view(np.uint8).reshape(-1, 16)
    assert (seen == 1).all(), "every packet finishes on exactly one rank"
    return out, ct, metrics, (pol[0], pol[1])
