"""Config 5 as ONE node across GPUs: endpoint-owned conntrack on the HIP datapath
(the CPU prototype of the protocol is tests/ep_shard.py).

The reference can give every endpoint its own CT maps: CT_MAP4 / CT_MAP6 are per-program
macros (bpf_lxc.c:53-75), per-endpoint maps when the endpoint's conntrack is local
(ConntrackLocal, pkg/endpoint/bpf.go:182-187).  Rank r owns the endpoints e with
e % world == r and their maps.  A packet's source program -- handle_ipv4_from_lxc /
ipv6_l3_from_lxc: the service lookup and lb{4,6}_local, the egress ct_lookup / ct_create,
the egress policy -- runs on its source's rank with the local delivery split off
(cv_lxc_egress_split); the delivery's 64-B record goes to the destination's rank, which
runs the destination's ipv4_policy / ipv6_policy on the destination's map
(cv_lxc_deliver).

Exact by construction: a CT map is touched only by its endpoint's source programs and by
deliveries into it, and an entry of it is keyed by the endpoint's address and one peer,
so every rank applies the operations of a map that share a peer in packet order; policy
counters and cilium_metrics are sums.  The candidate destinations of a packet and the
peers of its operations come from its headers and the read-only tables (`candidates`,
`peers`), as supersets; a source program that delivers anywhere else fails loudly.

A round: (1) the pending source operations that no earlier pending operation of their
map sharing a peer blocks, one split launch per family (the launch keeps a map's
operations in packet order: they share an address pair, so one group); (2) the
exchange: every candidate destination's owner gets the packet's record or a "not for
you" (one all_to_all of 72-B rows); (3) the deliveries now unblocked, one launch per
family, records in packet order.  Rounds repeat until no rank has pending operations.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence

import numpy as np

DEFER = -3                                     # CV_E_DEFER: a local delivery handed over
REC = 64                                       # delivery record bytes
ROW = 8 + REC                                  # exchange row: packet u32, destination u32, record
NONE_DST = 0xFFFFFFFF                          # a "not for you" resolution
FIELDS = ("ret", "reason", "identity", "ct", "proxy", "nl", "nu")


# ------------------------------------------------------------------ read-only node tables
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


def candidates(frames: np.ndarray, tables) -> List[frozenset]:
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


def peers(frames: np.ndarray, tables, loopback: int):
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


# ------------------------------------------------------------------ one rank
class EpNode:
    """One rank's endpoints, their maps (in `ctx`: every endpoint's CT4 / CT6 map its
    own) and their operations over one batch, in packet order.  frames / length / src_ep /
    flow_hash: the whole batch (host arrays; every rank holds it, each runs its part).
    exchange(rows_per_rank) -> rows from every rank: the collective (RCCL all_to_all at
    N > 1; see `dist_exchange`)."""

    def __init__(self, ctx, rank: int, world: int, frames: np.ndarray, length: np.ndarray, src_ep: np.ndarray,
                 flow_hash: np.ndarray, cand, src_p, dst_p, device="cuda:0", exchange=None, all_sum=None):
        import torch
        self.ctx, self.rank, self.world, self.dev = ctx, rank, world, device
        self.exchange = exchange or (lambda rows: [rows[0]])
        self.all_sum = all_sum or (lambda x: x)
        n = len(length)
        self.n = n
        self.cand = cand
        self.v6 = (frames[:, 12] == 0x86) & (frames[:, 13] == 0xDD)
        # the batch on the device, per family (64-B IPv4 / 128-B IPv6 records), as bench.py splits it
        self.rows = np.zeros(n, np.int64)
        self.fam = []
        for k, (sel, stride) in enumerate(((~self.v6, 64), (self.v6, 128))):
            idx = np.nonzero(sel)[0]
            self.rows[idx] = np.arange(len(idx))
            fr = np.ascontiguousarray(frames[idx, :stride]) if frames.shape[1] >= stride else \
                np.pad(frames[idx], ((0, 0), (0, stride - frames.shape[1])))
            self.fam.append({
                "frames": torch.from_numpy(np.ascontiguousarray(fr)).to(device),
                "length": torch.from_numpy(length[idx].astype(np.uint32).view(np.int32)).to(device),
                "src_ep": torch.from_numpy(src_ep[idx].astype(np.uint16).view(np.int16)).to(device),
                "flow_hash": torch.from_numpy(flow_hash[idx].astype(np.uint32).view(np.int32)).to(device)})
        # operations: (packet, kind 0 source / 1 delivery, map = endpoint) and their (map, peer) keys
        own = lambda e: e % world == rank
        op_pkt, op_kind, op_map, pr_op, pr_key = [], [], [], [], []
        keyid = {}
        for i in range(n):
            s = int(src_ep[i])
            todo = [(0, s, src_p[i])] if own(s) else []
            todo += [(1, d, dst_p[i]) for d in sorted(cand[i]) if own(d)]
            for kind, m, ps in todo:
                o = len(op_pkt)
                op_pkt.append(i)
                op_kind.append(kind)
                op_map.append(m)
                for pe in ps:
                    pr_op.append(o)
                    pr_key.append(keyid.setdefault((m, pe), len(keyid)))
        self.op_pkt = np.array(op_pkt, np.int64)
        self.op_kind = np.array(op_kind, np.int8)
        self.op_map = np.array(op_map, np.int64)
        self.op_order = self.op_pkt * 2 + self.op_kind
        self.pr_op = np.array(pr_op, np.int64)
        self.pr_key = np.array(pr_key, np.int64)
        self.nkeys = len(keyid)
        self.pending = np.ones(len(op_pkt), bool)
        self.resolved = self.op_kind == 0                          # deliveries: a record (or none) arrived
        self.record = {}                                           # delivery op -> its 64-B record
        self.op_of = {(int(p), int(m)): o for o, (p, k, m) in enumerate(zip(op_pkt, op_kind, op_map)) if k == 1}
        self.out = {k: np.zeros(n, np.int64) for k in FIELDS}
        self.mine = np.zeros(n, bool)                              # outputs final on this rank
        self.rounds = 0
        self.launches = 0
        self.cross = 0                                             # deliveries whose source ran on another rank

    # the candidates of `cand` that no earlier pending operation outside them blocks
    def _ready(self, cand: np.ndarray) -> np.ndarray:
        inc = cand.copy()
        while True:
            blocking = (self.pending & ~inc)[self.pr_op]
            blk = np.full(self.nkeys, np.iinfo(np.int64).max, np.int64)
            np.minimum.at(blk, self.pr_key[blocking], self.op_order[self.pr_op[blocking]])
            bad = inc[self.pr_op] & (self.op_order[self.pr_op] > blk[self.pr_key])
            if not bad.any():
                return inc
            inc[self.pr_op[bad]] = False

    def _host_out(self, out):
        import torch
        torch.cuda.synchronize()
        r = {k: v.cpu().numpy().astype(np.int64) for k, v in out.items()}
        r["identity"] &= 0xFFFFFFFF
        r["proxy"] &= 0xFFFF
        return r

    def _dev_out(self, m):
        import torch
        z = lambda dt: torch.zeros(m, dtype=dt, device=self.dev)
        return {"ret": z(torch.int32), "reason": z(torch.int32), "identity": z(torch.int32), "ct": z(torch.uint8),
                "proxy": z(torch.int16), "nl": z(torch.uint8), "nu": z(torch.uint8)}

    def _sources(self, pk: np.ndarray, now: int):
        """split launches of packets pk (sorted); returns the resolutions to send"""
        import torch
        res = []
        for k in (0, 1):
            sel = pk[self.v6[pk] == (k == 1)]
            if not len(sel):
                continue
            f = self.fam[k]
            r = torch.from_numpy(self.rows[sel]).to(self.dev)
            sub = {x: torch.index_select(t, 0, r).contiguous() for x, t in f.items()}
            out = self._dev_out(len(sel))
            dl = torch.zeros(len(sel) * REC, dtype=torch.uint8, device=self.dev)
            self.ctx.lxc_egress_split(sub["frames"], sub["length"], out, now, dl, src_ep=sub["src_ep"],
                                      flow_hash=sub["flow_hash"])
            self.launches += 1
            o = self._host_out(out)
            recs = dl.cpu().numpy().reshape(-1, REC)
            for j, i in enumerate(sel):
                i = int(i)
                dst = -1
                if o["ret"][j] == DEFER:
                    dst = int(recs[j, 48:50].view("<u2")[0] if k else recs[j, 24:26].view("<u2")[0])
                    if dst not in self.cand[i]:
                        raise RuntimeError(f"packet {i} delivered to endpoint {dst}, not a candidate "
                                           f"{sorted(self.cand[i])}")
                else:
                    for x in FIELDS:
                        self.out[x][i] = o[x][j]
                    self.mine[i] = True
                for d in self.cand[i] | ({dst} if dst >= 0 else set()):
                    res.append((i, d, recs[j] if d == dst else None))
        return res

    def _deliveries(self, ops: np.ndarray, now: int):
        import torch
        ops = ops[np.argsort(self.op_pkt[ops], kind="stable")]
        for k in (0, 1):
            sel = ops[self.v6[self.op_pkt[ops]] == (k == 1)]
            if not len(sel):
                continue
            recs = np.stack([self.record.pop(int(o)) for o in sel])
            rd = torch.from_numpy(np.ascontiguousarray(recs).reshape(-1)).to(self.dev)
            out = self._dev_out(len(sel))
            self.ctx.lxc_deliver(rd, len(sel), k == 1, out, now)
            self.launches += 1
            o = self._host_out(out)
            for j, op in enumerate(sel):
                i = int(self.op_pkt[op])
                for x in FIELDS:
                    self.out[x][i] = o[x][j]
                self.mine[i] = True

    def _receive(self, res):
        for i, d, rec in res:
            op = self.op_of[(int(i), int(d))]
            if rec is None:
                self.pending[op] = False                           # delivered elsewhere, or not at all
            else:
                self.record[op] = rec
            self.resolved[op] = True

    def run(self, now: int):
        """every operation of this rank; returns the rounds"""
        while True:
            left = self.all_sum(int(self.pending.sum()))
            if not left:
                return self.rounds
            self.rounds += 1
            before = int(self.pending.sum())
            # 1. the unblocked source programs
            src = self._ready(self.pending & (self.op_kind == 0))
            res = self._sources(np.sort(self.op_pkt[src]), now) if src.any() else []
            self.pending[src] = False
            # 2. every candidate's owner learns the record or "not for you"
            rows = [[] for _ in range(self.world)]
            for i, d, rec in res:
                rows[d % self.world].append((i, d, rec))
            got = self.exchange(rows)
            for r, rr in enumerate(got):
                if r != self.rank:
                    self.cross += sum(rec is not None for _, _, rec in rr)
                self._receive(rr)
            # 3. the unblocked deliveries
            dl = self._ready(self.pending & (self.op_kind == 1) & self.resolved)
            if dl.any():
                self._deliveries(np.nonzero(dl)[0], now)
                self.pending[dl] = False
            moved = self.all_sum(before - int(self.pending.sum()))
            if not moved:
                raise RuntimeError(f"rank {self.rank}: no operation could run in round {self.rounds}")


def dist_exchange(world: int, device: Optional[str] = None):
    """the round's exchange over torch.distributed: rows (packet, destination, 64-B record
    or "not for you") to every rank in one all_to_all_single of 72-B rows (RCCL with
    device tensors, gloo with host ones)"""
    import torch
    import torch.distributed as dist

    def pack(rows):
        a = np.zeros((len(rows), ROW), np.uint8)
        for j, (i, d, rec) in enumerate(rows):
            a[j, 0:4] = np.frombuffer(struct.pack("<I", i), np.uint8)
            a[j, 4:8] = np.frombuffer(struct.pack("<I", d if rec is not None else NONE_DST), np.uint8)
            if rec is not None:
                a[j, 8:] = rec
            else:                                                  # (the candidate, for the receiver)
                a[j, 8:12] = np.frombuffer(struct.pack("<I", d), np.uint8)
        return a

    def unpack(a):
        out = []
        for row in a.reshape(-1, ROW):
            i = int(row[0:4].view("<u4")[0])
            d = int(row[4:8].view("<u4")[0])
            if d == NONE_DST:
                out.append((i, int(row[8:12].view("<u4")[0]), None))
            else:
                out.append((i, d, row[8:].copy()))
        return out

    def exchange(rows_per_rank):
        parts = [pack(r) for r in rows_per_rank]
        cnt = torch.tensor([len(p) for p in parts], dtype=torch.int64, device=device)
        rcnt = torch.empty(world, dtype=torch.int64, device=device)
        dist.all_to_all_single(rcnt, cnt)
        send = torch.from_numpy(np.concatenate(parts).reshape(-1)).to(device) if sum(len(p) for p in parts) else \
            torch.zeros(0, dtype=torch.uint8, device=device)
        rsz = [int(x) * ROW for x in rcnt.cpu()]
        recv = torch.empty(sum(rsz), dtype=torch.uint8, device=device)
        dist.all_to_all_single(recv, send, rsz, [len(p) * ROW for p in parts])
        flat = recv.cpu().numpy()
        out, off = [], 0
        for sz in rsz:
            out.append(unpack(flat[off:off + sz]))
            off += sz
        return out

    def all_sum(x):
        t = torch.tensor([x], dtype=torch.int64, device=device)
        dist.all_reduce(t)
        return int(t.item())

    return exchange, all_sum
