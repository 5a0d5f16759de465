"""Deterministic synthetic workloads for the BASELINE.json configs.

Every table is produced as raw BPF key/value bytes (the exact layouts of
bpf/lib/common.h, bpf/lib/maps.h, bpf/lib/xdp.h) -- what the agent writes through
bpf(2) today (pkg/maps/*) -- so the product library and the CPU oracle are fed the
same bytes.  Packets are 64-B Ethernet/IPv4 frame records plus skb->len and
skb->mark arrays.  One SplitMix64 stream per config (seeds 0xC1A0_0001...).

Addresses are numpy uint32 in host integer form (10.0.0.1 == 0x0A000001) and are
written big-endian (network order) into keys and frames.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)

# BPF map types (include/linux/bpf.h)
MAP_HASH, MAP_LRU_HASH, MAP_LPM_TRIE = 1, 9, 11

# identities (bpf/node_config.h)
HOST_ID, WORLD_ID, CLUSTER_ID, HEALTH_ID = 1, 2, 3, 4

ETH_P_IP, ETH_P_ARP, ETH_P_IPV6 = 0x0800, 0x0806, 0x86DD
TCP, UDP, ICMP = 6, 17, 1
TCP_FIN, TCP_SYN, TCP_RST, TCP_PSH, TCP_ACK = 0x01, 0x02, 0x04, 0x08, 0x10


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


class Stream:
    """A SplitMix64 stream consumed in order."""

    def __init__(self, seed: int):
        self.seed = seed & ((1 << 64) - 1)
        self.pos = 0

    def u64(self, n: int) -> np.ndarray:
        out = splitmix64(self.seed, n, self.pos)
        self.pos += n
        return out

    def u32(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(32)).astype(np.uint32)

    def randint(self, n: int, lo: int, hi: int) -> np.ndarray:
        """uniform integers in [lo, hi)"""
        return (self.u64(n) % np.uint64(hi - lo)).astype(np.int64) + lo

    def frac(self, n: int) -> np.ndarray:
        return (self.u64(n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))

    def choice(self, n: int, k: int) -> np.ndarray:
        return self.randint(n, 0, k)


@dataclasses.dataclass
class MapSpec:
    """A BPF map as the agent would create and fill it."""
    name: str
    type: int
    key_size: int
    val_size: int
    max_entries: int
    keys: np.ndarray          # (n, key_size) uint8, insertion order
    vals: np.ndarray          # (n, val_size) uint8

    def __len__(self):
        return len(self.keys)


@dataclasses.dataclass
class Workload:
    name: str
    maps: Dict[str, MapSpec]
    frames: np.ndarray        # (n, stride) uint8
    length: np.ndarray        # (n,) uint32  skb->len
    mark: np.ndarray          # (n,) uint32  skb->mark
    endpoints: List[dict]     # per local endpoint: lxc_id, seclabel, ip, ifindex
    now: int = 0
    extra: Optional[dict] = None

    @property
    def n(self) -> int:
        return len(self.length)


def be32_bytes(a: np.ndarray) -> np.ndarray:
    return a.astype(">u4").view(np.uint8).reshape(-1, 4)


def be16_bytes(a: np.ndarray) -> np.ndarray:
    return a.astype(">u2").view(np.uint8).reshape(-1, 2)


def le32_bytes(a: np.ndarray) -> np.ndarray:
    return a.astype("<u4").view(np.uint8).reshape(-1, 4)


def le16_bytes(a: np.ndarray) -> np.ndarray:
    return a.astype("<u2").view(np.uint8).reshape(-1, 2)


def prefix_mask(plen: np.ndarray) -> np.ndarray:
    plen = np.asarray(plen, dtype=np.int64)
    m = np.where(plen <= 0, 0, (0xFFFFFFFF << (32 - np.clip(plen, 1, 32))) & 0xFFFFFFFF)
    return m.astype(np.uint32)


# --------------------------------------------------------------------------
# key / value builders (layouts: SURVEY.md Appendix A)
# --------------------------------------------------------------------------

def lpm_v4_keys(addr: np.ndarray, plen: np.ndarray) -> np.ndarray:
    """struct lpm_v4_key (bpf/lib/xdp.h:23-26): u32 prefixlen + 4 address bytes."""
    k = np.zeros((len(addr), 8), np.uint8)
    k[:, 0:4] = le32_bytes(np.asarray(plen, np.uint32))
    k[:, 4:8] = be32_bytes(addr)
    return k


def endpoint_keys_v4(ip: np.ndarray) -> np.ndarray:
    """struct endpoint_key (bpf/lib/common.h:147-160), family 1."""
    k = np.zeros((len(ip), 20), np.uint8)
    k[:, 0:4] = be32_bytes(ip)
    k[:, 16] = 1
    return k


def endpoint_infos(ifindex, lxc_id, flags) -> np.ndarray:
    """struct endpoint_info (bpf/lib/common.h:165-173), 48 bytes."""
    n = len(lxc_id)
    v = np.zeros((n, 48), np.uint8)
    v[:, 0:4] = le32_bytes(np.asarray(ifindex, np.uint32))
    v[:, 6:8] = le16_bytes(np.asarray(lxc_id, np.uint16))
    v[:, 8:12] = le32_bytes(np.asarray(flags, np.uint32))
    v[:, 16:22] = np.array([0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF], np.uint8)
    v[:, 24:30] = np.array([0xDE, 0xAD, 0xBE, 0xEF, 0xC0, 0xDE], np.uint8)
    return v


def ipcache_keys_v4(addr: np.ndarray, plen: np.ndarray) -> np.ndarray:
    """struct ipcache_key (bpf/lib/maps.h:135-148): prefixlen = 32 static bits + CIDR."""
    k = np.zeros((len(addr), 24), np.uint8)
    k[:, 0:4] = le32_bytes(np.asarray(plen, np.uint32) + 32)
    k[:, 7] = 1
    k[:, 8:12] = be32_bytes(addr)
    return k


def remote_endpoint_infos(sec_label, tunnel=None) -> np.ndarray:
    n = len(sec_label)
    v = np.zeros((n, 8), np.uint8)
    v[:, 0:4] = le32_bytes(np.asarray(sec_label, np.uint32))
    if tunnel is not None:
        v[:, 4:8] = be32_bytes(np.asarray(tunnel, np.uint32))
    return v


def policy_keys(identity, dport, proto, egress=0) -> np.ndarray:
    """struct policy_key (bpf/lib/common.h:180-186); dport in network order."""
    n = len(identity)
    k = np.zeros((n, 8), np.uint8)
    k[:, 0:4] = le32_bytes(np.asarray(identity, np.uint32))
    k[:, 4:6] = be16_bytes(np.asarray(dport, np.uint16))
    k[:, 6] = np.asarray(proto, np.uint8)
    k[:, 7] = np.uint8(1 if egress else 0)
    return k


def policy_entries(proxy_port) -> np.ndarray:
    """struct policy_entry (bpf/lib/common.h:188-193); proxy_port network order."""
    n = len(proxy_port)
    v = np.zeros((n, 24), np.uint8)
    v[:, 0:2] = be16_bytes(np.asarray(proxy_port, np.uint16))
    return v


# --------------------------------------------------------------------------
# frames
# --------------------------------------------------------------------------

def ipv4_frames(saddr, daddr, proto, sport, dport, tcp_flags, ttl, ethertype=None,
                stride: int = 64, icmp_type=None) -> np.ndarray:
    """Ethernet + IPv4 (ihl 5) + L4 header records of `stride` bytes."""
    n = len(saddr)
    f = np.zeros((n, stride), np.uint8)
    f[:, 0:6] = np.array([0xDE, 0xAD, 0xBE, 0xEF, 0xC0, 0xDE], np.uint8)   # NODE_MAC
    f[:, 6:12] = np.array([0x02, 0x00, 0x00, 0x00, 0x00, 0x01], np.uint8)
    et = np.full(n, ETH_P_IP, np.uint16) if ethertype is None else np.asarray(ethertype, np.uint16)
    f[:, 12:14] = be16_bytes(et)
    f[:, 14] = 0x45
    f[:, 16:18] = be16_bytes(np.full(n, stride - 14, np.uint16))
    f[:, 22] = np.asarray(ttl, np.uint8)
    proto = np.asarray(proto, np.uint8)
    f[:, 23] = proto
    f[:, 26:30] = be32_bytes(saddr)
    f[:, 30:34] = be32_bytes(daddr)
    l4 = 34
    isports = (proto == TCP) | (proto == UDP)
    sp = be16_bytes(np.asarray(sport, np.uint16))
    dp = be16_bytes(np.asarray(dport, np.uint16))
    f[isports, l4:l4 + 2] = sp[isports]
    f[isports, l4 + 2:l4 + 4] = dp[isports]
    tcp = proto == TCP
    f[tcp, l4 + 12] = 0x50                                   # data offset 5
    f[tcp, l4 + 13] = np.asarray(tcp_flags, np.uint8)[tcp]
    icmp = proto == ICMP
    if icmp_type is not None:
        f[icmp, l4] = np.asarray(icmp_type, np.uint8)[icmp]
    return f


def _rand_addrs_in(stream: Stream, base: np.ndarray, plen: np.ndarray) -> np.ndarray:
    host = stream.u32(len(base)) & ~prefix_mask(plen)
    return (base & prefix_mask(plen)) | host


# --------------------------------------------------------------------------
# Config 1: bpf_xdp.c CIDR prefilter (1k prefixes, 1M headers)
# --------------------------------------------------------------------------

def config1(n_pkts: int = 1 << 20, seed: int = 0xC1A00001, n_fix: int = 256, n_dyn: int = 768,
            n_ep: int = 4096, n_host: int = 4) -> Workload:
    s = Stream(seed)
    fix = s.u32(n_fix)
    dyn_len = s.randint(n_dyn, 8, 32)
    dyn = s.u32(n_dyn) & prefix_mask(dyn_len)
    # endpoints: distinct IPs in 10.0.0.0/16
    ep_host = np.unique(s.randint(n_ep * 2, 1, 65535).astype(np.uint32))[:n_ep]
    ep_ip = np.uint32(0x0A000000) | ep_host
    host_ip = np.uint32(0x0A010000) | np.arange(1, n_host + 1, dtype=np.uint32)
    lxc_ip = np.concatenate([ep_ip, host_ip])
    lxc_id = np.concatenate([np.arange(1, len(ep_ip) + 1), np.zeros(n_host)]).astype(np.uint16)
    lxc_flags = np.concatenate([np.zeros(len(ep_ip)), np.ones(n_host)]).astype(np.uint32)
    ifindex = np.concatenate([np.arange(100, 100 + len(ep_ip)), np.zeros(n_host)]).astype(np.uint32)
    maps = {
        "v4_fix": MapSpec("cilium_cidr_v4_fix", MAP_HASH, 8, 1, 1 << 20,
                          lpm_v4_keys(fix, np.full(n_fix, 32)), np.zeros((n_fix, 1), np.uint8)),
        "v4_dyn": MapSpec("cilium_cidr_v4_dyn", MAP_LPM_TRIE, 8, 1, 1 << 16,
                          lpm_v4_keys(dyn, dyn_len), np.zeros((n_dyn, 1), np.uint8)),
        "lxc": MapSpec("cilium_lxc", MAP_HASH, 20, 48, 65536, endpoint_keys_v4(lxc_ip),
                       endpoint_infos(ifindex, lxc_id, lxc_flags)),
    }
    # packets
    in_deny = s.frac(n_pkts) < 0.5
    pick = s.choice(n_pkts, n_fix + n_dyn)
    bases = np.concatenate([fix, dyn])[pick]
    plens = np.concatenate([np.full(n_fix, 32), dyn_len])[pick]
    saddr = np.where(in_deny, _rand_addrs_in(s, bases, plens), s.u32(n_pkts))
    to_ep = s.frac(n_pkts) < 0.8
    daddr = np.where(to_ep, lxc_ip[s.choice(n_pkts, len(lxc_ip))], s.u32(n_pkts))
    sport = s.randint(n_pkts, 1024, 65536)
    dport = s.randint(n_pkts, 1, 65536)
    r = s.frac(n_pkts)
    ethertype = np.where(r < 0.01, ETH_P_ARP, ETH_P_IP)
    frames = ipv4_frames(saddr, daddr, np.full(n_pkts, TCP), sport, dport,
                         np.full(n_pkts, TCP_ACK), np.full(n_pkts, 64), ethertype)
    length = np.full(n_pkts, 64, np.uint32)
    short = s.frac(n_pkts) < 0.001
    length[short] = s.randint(int(short.sum()), 14, 34).astype(np.uint32)
    return Workload("config1", maps, frames, length, np.zeros(n_pkts, np.uint32), [],
                    extra={"lxc_ip": lxc_ip})


# --------------------------------------------------------------------------
# Config 2: ipcache LPM (100k CIDRs) + policymap (10k identities x L4) ingress
# --------------------------------------------------------------------------

def config2(n_pkts: int = 1 << 20, seed: int = 0xC1A00002, n_cidrs: int = 102400,
            n_ids: int = 10000, l4_per_id: int = 8, n_wild: int = 64) -> Workload:
    s = Stream(seed)
    # ipcache CIDRs: 70% /32, 25% /24-/31, 5% /8-/23, plus 0.0.0.0/0 -> WORLD
    n32 = int(n_cidrs * 0.70)
    n24 = int(n_cidrs * 0.25)
    n8 = n_cidrs - n32 - n24
    plen = np.concatenate([np.full(n32, 32), s.randint(n24, 24, 32), s.randint(n8, 8, 24)])
    addr = s.u32(n_cidrs) & prefix_mask(plen)
    ids = np.arange(256, 256 + n_ids, dtype=np.uint32)
    ident = ids[s.choice(n_cidrs, n_ids)]
    ip_addr = np.concatenate([addr, np.zeros(1, np.uint32)])
    ip_plen = np.concatenate([plen, np.zeros(1)])
    ip_ident = np.concatenate([ident, np.full(1, WORLD_ID, np.uint32)])
    ipcache = MapSpec("cilium_ipcache", MAP_LPM_TRIE, 24, 8, 512000,
                      ipcache_keys_v4(ip_addr, ip_plen), remote_endpoint_infos(ip_ident))

    # policy for one endpoint (ingress)
    port_pool = np.unique(np.concatenate([[80, 443, 53, 8080], s.randint(200, 1, 65536)]))[:64]
    combos_p = np.stack(np.meshgrid(port_pool, [TCP, UDP], indexing="ij"), -1).reshape(-1, 2)
    wild_ports = np.setdiff1d(np.unique(s.randint(512, 1, 65536)), port_pool)[:128]
    combos_w = np.stack(np.meshgrid(wild_ports, [TCP, UDP], indexing="ij"), -1).reshape(-1, 2)
    # per identity: l4_per_id distinct combos out of combos_p
    sel = np.argsort(s.u64(n_ids * len(combos_p)).reshape(n_ids, len(combos_p)), axis=1)[:, :l4_per_id]
    c = combos_p[sel].reshape(-1, 2)
    pol_id = np.repeat(ids, l4_per_id)
    pol_port, pol_proto = c[:, 0], c[:, 1]
    l3 = ids[s.frac(n_ids) < 0.10]
    wsel = np.argsort(s.u64(len(combos_w)))[:n_wild]
    wild = combos_w[wsel]
    k_id = np.concatenate([pol_id, l3, np.zeros(n_wild, np.uint32)])
    k_port = np.concatenate([pol_port, np.zeros(len(l3)), wild[:, 0]])
    k_proto = np.concatenate([pol_proto, np.zeros(len(l3)), wild[:, 1]])
    nk = len(k_id)
    proxy = np.where(s.frac(nk) < 0.05, s.randint(nk, 10000, 20000), 0)
    policy = MapSpec("cilium_policy_1", MAP_HASH, 8, 24, max(16384, 1 << int(np.ceil(np.log2(nk * 1.25)))),
                     policy_keys(k_id, k_port, k_proto), policy_entries(proxy))

    ep_ip = np.array([0x0A00000A], np.uint32)
    lxc = MapSpec("cilium_lxc", MAP_HASH, 20, 48, 65536, endpoint_keys_v4(ep_ip),
                  endpoint_infos([7], [1], [0]))

    # packets: saddr 90% inside ipcache CIDRs; dport 70% from the ports the source
    # identity is allowed on (its L4 entries), else wildcard / uniform ports
    inside = s.frac(n_pkts) < 0.90
    pick = s.choice(n_pkts, n_cidrs)
    saddr = np.where(inside, _rand_addrs_in(s, addr[pick], plen[pick]), s.u32(n_pkts))
    id_idx = ident[pick] - 256
    own = combos_p[sel[id_idx, s.choice(n_pkts, l4_per_id)]]
    wild_c = combos_w[s.choice(n_pkts, len(combos_w))]
    r = s.frac(n_pkts)
    use_own = inside & (r < 0.70)
    use_wild = ~use_own & (r < 0.85)
    dport = np.where(use_own, own[:, 0], np.where(use_wild, wild_c[:, 0], s.randint(n_pkts, 1, 65536)))
    proto = np.where(use_own, own[:, 1], np.where(use_wild, wild_c[:, 1], TCP)).astype(np.uint8)
    r = s.frac(n_pkts)
    proto = np.where(~use_own & ~use_wild, np.where(r < 0.6, TCP, np.where(r < 0.95, UDP, ICMP)),
                     proto).astype(np.uint8)
    sport = s.randint(n_pkts, 1024, 65536)
    icmp_type = np.where(s.frac(n_pkts) < 0.5, 8, 0)
    flags = np.full(n_pkts, TCP_ACK)
    frames = ipv4_frames(saddr, np.full(n_pkts, ep_ip[0]), proto, sport, dport, flags,
                         np.full(n_pkts, 64), icmp_type=icmp_type)
    return Workload("config2", {"ipcache": ipcache, "policy": policy, "lxc": lxc}, frames,
                    np.full(n_pkts, 64, np.uint32), np.zeros(n_pkts, np.uint32),
                    [{"lxc_id": 1, "seclabel": 0x1010, "ip": int(ep_ip[0]), "ifindex": 7}])


# --------------------------------------------------------------------------
# Config 3: full bpf_lxc ingress path: prefilter + ipcache + lxc + policy + CT
# --------------------------------------------------------------------------

def ct4_keys(daddr, saddr, dport, sport, nexthdr, flags) -> np.ndarray:
    """struct ipv4_ct_tuple (bpf/lib/common.h:359-367), packed 14 bytes."""
    n = len(daddr)
    k = np.zeros((n, 14), np.uint8)
    k[:, 0:4] = be32_bytes(daddr)
    k[:, 4:8] = be32_bytes(saddr)
    k[:, 8:10] = be16_bytes(np.asarray(dport, np.uint16))
    k[:, 10:12] = be16_bytes(np.asarray(sport, np.uint16))
    k[:, 12] = np.asarray(nexthdr, np.uint8)
    k[:, 13] = np.asarray(flags, np.uint8)
    return k


def ct_entries(n, now, ingress, tcp, src_sec_id, seen_non_syn=False, length=64) -> np.ndarray:
    """struct ct_entry (bpf/lib/common.h:380-406), 56 bytes: an established entry
    as an agent restore would write it (counters of one packet, lifetime now+60/21600)."""
    v = np.zeros((n, 56), np.uint8)
    ingress = np.asarray(ingress, bool)
    tcp = np.asarray(tcp, bool)
    one = np.ones(n, np.uint64)
    ln = np.full(n, length, np.uint64)
    rx = np.where(ingress, one, 0).astype("<u8")
    tx = np.where(ingress, 0, one).astype("<u8")
    v[:, 0:8] = rx.view(np.uint8).reshape(n, 8)
    v[:, 8:16] = np.where(ingress, ln, 0).astype("<u8").view(np.uint8).reshape(n, 8)
    v[:, 16:24] = tx.view(np.uint8).reshape(n, 8)
    v[:, 24:32] = np.where(ingress, 0, ln).astype("<u8").view(np.uint8).reshape(n, 8)
    life = np.where(tcp & ~np.asarray(seen_non_syn, bool), 60, np.where(tcp, 21600, 60)) + now
    v[:, 32:36] = le32_bytes(life.astype(np.uint32))
    bits = np.where(np.asarray(seen_non_syn, bool), 0x10, 0).astype(np.uint16)
    v[:, 36:38] = le16_bytes(bits)
    fl = np.where(tcp, TCP_SYN, 0).astype(np.uint8)
    v[:, 42] = np.where(ingress, 0, fl)          # tx_flags_seen
    v[:, 43] = np.where(ingress, fl, 0)          # rx_flags_seen
    v[:, 44:48] = le32_bytes(np.asarray(src_sec_id, np.uint32))
    v[:, 48:52] = le32_bytes(np.where(ingress, 0, now).astype(np.uint32))   # last_tx_report
    v[:, 52:56] = le32_bytes(np.where(ingress, now, 0).astype(np.uint32))   # last_rx_report
    return v


def zipf_ranks(s: "Stream", n: int, N: int, a: float) -> np.ndarray:
    """n draws from a Zipf(a) popularity over N items (P(rank k) ~ (k + 1)^-a, the
    continuous inverse CDF), mapped through a fixed bijection of [0, N) so the popular
    items are scattered over the table rather than its first rows."""
    u = s.frac(n)
    if abs(a - 1.0) < 1e-9:
        x = np.exp(u * np.log(N + 1.0))
    else:
        x = ((np.power(N + 1.0, 1.0 - a) - 1.0) * u + 1.0) ** (1.0 / (1.0 - a))
    r = np.clip(np.floor(x).astype(np.int64) - 1, 0, N - 1)
    mult = 0x9E3779B1
    while np.gcd(mult, N) != 1:
        mult += 2
    return ((r.astype(np.uint64) * np.uint64(mult) + np.uint64(12345)) % np.uint64(N)).astype(np.int64)


def config3(n_pkts: int = 1 << 24, n_flows: int = 1 << 24, seed: int = 0xC1A00003, now0: int = 1_000_000,
            n_cidrs: int = 102400, n_ids: int = 10000, n_ep: int = 4096, ct_max: Optional[int] = None,
            ttl_low: float = 0.0005, v6_frac: float = 0.0, stride: Optional[int] = None,
            n_flows6: Optional[int] = None, shard: Optional[Tuple[int, int]] = None,
            zipf: Optional[float] = None, ep_zipf: Optional[float] = None) -> Workload:
    """Ingress through from_netdev into the endpoints' policy programs with conntrack.
    v6_frac > 0 makes a dual-stack batch: that fraction of the packets becomes IPv6
    (handle_ipv6 -> ipv6_policy with a global CT6 map, v6 endpoints in cilium_lxc, v6
    ipcache entries), drawn after every IPv4 draw so the IPv4 part is unchanged;
    records are then 128 bytes unless `stride` says otherwise.
    shard = (rank, world): config 4, rank's part of ONE node-wide flow set: every rank
    draws the same candidate (remote, endpoint) pairs from the same seed and keeps
    those whose address pair (cilium_amd.shard.pair_key4) it owns, n_flows of them; its
    packets (existing and new flows) are its own pairs too, as a producer steering by
    address pair would hand them over.  The ranks' CT shards are disjoint.
    zipf = a: the existing flows' packets (forward and reply) follow a Zipf(a) popularity
    instead of a uniform one (elephant flows: a few address pairs carry many packets of
    the batch); drawn from a stream of their own, the rest of the batch is unchanged.
    ep_zipf = a: the existing flows' local endpoints follow Zipf(a) instead of a uniform
    draw (a few endpoints hold most connections: with per-endpoint CT maps,
    per_endpoint_ct, their maps are the ones at max_entries)."""
    s = Stream(seed)
    c1 = config1(16, n_ep=n_ep)
    c2 = config2(16, n_cidrs=n_cidrs, n_ids=n_ids)
    maps = {k: c1.maps[k] for k in ("v4_fix", "v4_dyn", "lxc")}
    maps["ipcache"] = c2.maps["ipcache"]
    maps["policy"] = c2.maps["policy"]
    lxc_ip = c1.extra["lxc_ip"][:n_ep]                   # endpoints (not the host IPs)
    ep_ids = np.arange(1, n_ep + 1)
    # flows: remote (inside an ipcache CIDR) <-> endpoint
    ipk = c2.maps["ipcache"].keys[:-1]
    cidr_addr = ipk[:, 8:12].copy().view(">u4").reshape(-1).astype(np.uint32)
    cidr_plen = ipk[:, 0:4].copy().view("<u4").reshape(-1).astype(np.int64) - 32
    if shard is None or shard[1] <= 1:
        pick = s.choice(n_flows, len(cidr_addr))
        remote = _rand_addrs_in(s, cidr_addr[pick], cidr_plen[pick])
        epi = s.choice(n_flows, n_ep)
        if ep_zipf:
            epi = zipf_ranks(Stream(seed ^ 0xE9E9E9E9), n_flows, n_ep, ep_zipf)
    else:
        pick, remote, epi = _owned_pairs(s, n_flows, shard, cidr_addr, cidr_plen, lxc_ip)
    local = lxc_ip[epi]
    pol = c2.maps["policy"].keys
    pol_port = pol[:, 4:6].copy().view(">u2").reshape(-1)
    pol_proto = pol[:, 6]
    l4 = pol_proto != 0
    pp, pr = pol_port[l4], pol_proto[l4]
    ident = c2.maps["ipcache"].vals[pick, 0:4].copy().view("<u4").reshape(-1)
    # a connection exists because the policy let it in: the service port is one the
    # remote's identity may reach (its L4 entries; an identity without any: a random one)
    sel = s.choice(n_flows, len(pp))
    aport, aproto, has = _allowed_l4(pol, ident, s)
    fport = np.where(has, aport, pp[sel]).astype(np.int64)
    fproto = np.where(has, aproto, pr[sel]).astype(np.uint8)
    eport = s.randint(n_flows, 1024, 65536)
    ingress_init = s.frac(n_flows) < 0.75
    # CT entries: ingress-initiated {daddr remote, saddr local, dport fport, sport eport, IN}
    #             egress-initiated  {daddr local, saddr remote, dport fport(remote), sport eport(local), OUT}
    d_addr = np.where(ingress_init, remote, local)
    s_addr = np.where(ingress_init, local, remote)
    keys = ct4_keys(d_addr, s_addr, fport, eport, fproto, np.where(ingress_init, 1, 0))
    tcp = fproto == TCP
    seclabel = (0x1000 + ep_ids[epi]).astype(np.uint32)
    vals = ct_entries(n_flows, now0, ingress_init, tcp, np.where(ingress_init, ident, seclabel),
                      seen_non_syn=tcp)
    # ICMP-related twins (conntrack.h:727-741): one per address pair, last writer wins
    rk = ct4_keys(d_addr, s_addr, np.zeros(n_flows), np.zeros(n_flows), np.full(n_flows, ICMP),
                  np.where(ingress_init, 3, 2))
    rv = vals.copy()
    rv[:, 36] |= 0x10
    all_k = np.concatenate([keys, rk])
    all_v = np.concatenate([vals, rv])
    cap = ct_max or max(1 << 20, 1 << int(np.ceil(np.log2(len(all_k) * 1.25))))
    maps["ct4"] = MapSpec("cilium_ct4_global", MAP_LRU_HASH, 14, 56, cap, all_k, all_v)
    # packets: 60% existing forward (ingress-initiated), 20% reply (egress-initiated), 20% new
    r = s.frac(n_pkts)
    ing_idx = np.nonzero(ingress_init)[0]
    egr_idx = np.nonzero(~ingress_init)[0]
    fi = ing_idx[s.choice(n_pkts, len(ing_idx))]
    fe = egr_idx[s.choice(n_pkts, max(len(egr_idx), 1))] if len(egr_idx) else fi
    if zipf:
        zs = Stream(seed ^ 0x5A1F5A1F)
        fi = ing_idx[zipf_ranks(zs, n_pkts, len(ing_idx), zipf)]
        fe = egr_idx[zipf_ranks(zs, n_pkts, len(egr_idx), zipf)] if len(egr_idx) else fi
    kind = np.where(r < 0.6, 0, np.where(r < 0.8, 1, 2))
    f = np.where(kind == 0, fi, fe)
    saddr = remote[f].copy()
    daddr = local[f].copy()
    sport = np.where(kind == 0, eport[f], fport[f])
    dport = np.where(kind == 0, fport[f], eport[f])
    proto = fproto[f].copy()
    new = kind == 2
    nn = int(new.sum())
    if shard is None or shard[1] <= 1:
        npk = s.choice(nn, len(cidr_addr))
        saddr[new] = _rand_addrs_in(s, cidr_addr[npk], cidr_plen[npk])
        daddr[new] = lxc_ip[s.choice(nn, n_ep)]
    else:
        npk, nrem, nepi = _owned_pairs(s, nn, shard, cidr_addr, cidr_plen, lxc_ip)
        saddr[new] = nrem
        daddr[new] = lxc_ip[nepi]
    sport[new] = s.randint(nn, 1024, 65536)
    nsel = s.choice(nn, len(pp))
    nid = c2.maps["ipcache"].vals[npk, 0:4].copy().view("<u4").reshape(-1)
    nport, nproto, nhas = _allowed_l4(pol, nid, s)
    r2 = s.frac(nn)                                     # 70% to a port the policy allows
    allow = nhas & (r2 < 0.7)
    dport[new] = np.where(allow, nport, np.where(r2 < 0.85, pp[nsel], s.randint(nn, 1, 65536)))
    proto[new] = np.where(allow, nproto, pr[nsel])
    rf = s.frac(n_pkts)
    flags = np.where(rf < 0.90, TCP_ACK, np.where(rf < 0.95, TCP_SYN, np.where(rf < 0.98, TCP_FIN | TCP_ACK, TCP_RST)))
    ttl = np.where(s.frac(n_pkts) < ttl_low, 1, 64)
    frames = ipv4_frames(saddr, daddr, proto, sport, dport, flags, ttl)
    eps = [{"lxc_id": int(i), "seclabel": int(0x1000 + i), "ip": int(lxc_ip[i - 1])} for i in ep_ids]
    length = np.full(n_pkts, 64, np.uint32)
    extra = {"kind": kind, "node": {"router_ip6": ROUTER_IP6, "host_mac": bytes(HOST_IFINDEX_MAC),
                                    "net_mac": bytes(CILIUM_NET_MAC)}}
    if v6_frac > 0:
        stride = stride or 128
        f6 = np.zeros((n_pkts, stride), np.uint8)
        f6[:, :64] = frames
        frames = f6
        v6 = _config3_v6(s, maps, c2, frames, length, kind, eps, v6_frac, n_flows6 or max(n_flows // 4, 16), n_ep,
                         now0, ct_max, pp, pr)
        extra["v6"] = v6
    elif stride and stride > 64:
        f6 = np.zeros((n_pkts, stride), np.uint8)
        f6[:, :64] = frames
        frames = f6
    return Workload("config3", maps, frames, length, np.zeros(n_pkts, np.uint32), eps, now=now0 + 1, extra=extra)


HOST_IFINDEX_MAC = np.array([0xCE, 0x72, 0xA7, 0x03, 0x88, 0x56], np.uint8)    # bpf/node_config.h:39
CILIUM_NET_MAC = np.array([0xCE, 0x72, 0xA7, 0x03, 0x88, 0x57], np.uint8)      # bpf/node_config.h:57


def ct6_keys(daddr6, saddr6, dport, sport, nexthdr, flags) -> np.ndarray:
    """struct ipv6_ct_tuple (bpf/lib/common.h:338-346), 40 bytes with 2 zero pad bytes."""
    n = len(daddr6)
    k = np.zeros((n, 40), np.uint8)
    k[:, 0:16] = daddr6
    k[:, 16:32] = saddr6
    k[:, 32:34] = be16_bytes(np.asarray(dport, np.uint16))
    k[:, 34:36] = be16_bytes(np.asarray(sport, np.uint16))
    k[:, 36] = np.asarray(nexthdr, np.uint8)
    k[:, 37] = np.asarray(flags, np.uint8)
    return k


def _owned_pairs(s, n, shard, cidr_addr, cidr_plen, lxc_ip, chunk=1 << 22):
    """n (CIDR index, remote address, endpoint index) candidates, drawn in order from
    stream s, whose (remote, endpoint) address pair belongs to shard = (rank, world).
    Every rank consumes the same candidate sequence, so the kept sets are disjoint
    parts of one flow set."""
    from cilium_amd.shard import pair_key4
    rank, world = shard
    picks, rems, epis, got = [], [], [], 0
    while got < n:
        pick = s.choice(chunk, len(cidr_addr))
        rem = _rand_addrs_in(s, cidr_addr[pick], cidr_plen[pick])
        epi = s.choice(chunk, len(lxc_ip))
        raw = lambda a: a.astype(np.uint32).byteswap()              # the frame's raw word
        own = (pair_key4(raw(rem), raw(lxc_ip[epi])) % np.uint64(world)) == np.uint64(rank)
        picks.append(pick[own]); rems.append(rem[own]); epis.append(epi[own])
        got += int(own.sum())
    return (np.concatenate(picks)[:n], np.concatenate(rems)[:n], np.concatenate(epis)[:n])


def _allowed_l4(pol_keys, ident, s):
    """Per identity of `ident`: one (dport, proto) of its ingress L4 policy entries
    (policy_key rows), chosen uniformly; `has` false where it has none."""
    pid = pol_keys[:, 0:4].copy().view("<u4").reshape(-1)
    port = pol_keys[:, 4:6].copy().view(">u2").reshape(-1).astype(np.int64)
    proto = pol_keys[:, 6]
    ok = (pid != 0) & (proto != 0) & (pol_keys[:, 7] == 0)
    order = np.argsort(pid[ok], kind="stable")
    ids, ports, protos = pid[ok][order], port[ok][order], proto[ok][order]
    lo = np.searchsorted(ids, ident, "left")
    cnt = np.searchsorted(ids, ident, "right") - lo
    r = (s.u64(len(ident)) % np.maximum(cnt, 1).astype(np.uint64)).astype(np.int64)
    at = np.minimum(lo + r, max(len(ids) - 1, 0))
    has = cnt > 0
    if not len(ids):
        return np.zeros(len(ident), np.int64), np.zeros(len(ident), np.uint8), has
    return ports[at], protos[at], has


def _config3_v6(s, maps, c2, frames, length, kind4, eps, v6_frac, n_flows6, n_ep, now0, ct_max, pp, pr):
    """The IPv6 half of a dual-stack config 3 (see config3): tables and packets."""
    n_pkts = len(length)
    ep_idx = np.arange(n_ep)
    ep_ip6 = v6_addrs(V6_POD_PREFIX, np.full(n_ep, 0x000A0000), (ep_idx + 0x100).astype(np.uint32) * 0x10001)
    for e, a in zip(eps, ep_ip6):
        e["ip6"] = bytes(a)
    # cilium_lxc: the v6 endpoint addresses (same lxc ids / ifindexes) + the router as HOST
    lk = maps["lxc"]
    k6 = np.concatenate([endpoint_keys_v6(ep_ip6), endpoint_keys_v6(np.frombuffer(ROUTER_IP6, np.uint8)[None])])
    v6v = np.concatenate([lk.vals[:n_ep], endpoint_infos([0], [0], [1])])
    maps["lxc"] = MapSpec(lk.name, lk.type, 20, 48, lk.max_entries, np.concatenate([lk.keys, k6]),
                          np.concatenate([lk.vals, v6v]))
    # ipcache: remote v6 pods /128 and a few /64s -> identities of the config-2 id space
    n_r6 = 4096
    remote6 = v6_addrs(bytes([0x20, 0x01, 0x0D, 0xB8, 0, 0, 0, 7]), np.zeros(n_r6), np.arange(n_r6, dtype=np.uint32) + 1)
    r_id = (256 + s.choice(n_r6, 10000)).astype(np.uint32)
    nets = v6_addrs(bytes([0x20, 0x01, 0x0D, 0xB8, 0, 0, 0, 0]), np.zeros(64), np.zeros(64))
    nets[:, 6:8] = be16_bytes(np.arange(64, dtype=np.uint16) + 0x100)
    n_id = (256 + s.choice(64, 10000)).astype(np.uint32)
    ik = c2.maps["ipcache"] if "ipcache" not in maps else maps["ipcache"]
    maps["ipcache"] = MapSpec(ik.name, ik.type, 24, 8, ik.max_entries,
                              np.concatenate([ik.keys, ipcache_keys_v6(remote6, np.full(n_r6, 128)),
                                              ipcache_keys_v6(nets, np.full(64, 64))]),
                              np.concatenate([ik.vals, remote_endpoint_infos(np.concatenate([r_id, n_id]))]))
    # flows: remote (a /128 pod or an address in a /64) <-> local endpoint, CT6 preloaded
    F = n_flows6
    in_net = s.frac(F) < 0.3
    ri = s.choice(F, n_r6)
    ni = s.choice(F, 64)
    rem = remote6[ri].copy()
    netp = nets[ni].copy()
    netp[:, 8:16] = s.u64(F).astype(">u8").view(np.uint8).reshape(F, 8)
    rem = np.where(in_net[:, None], netp, rem)
    epi = s.choice(F, n_ep)
    loc = ep_ip6[epi]
    sel = s.choice(F, len(pp))
    pol = c2.maps["policy"].keys
    aport, aproto, has = _allowed_l4(pol, np.where(in_net, n_id[ni], r_id[ri]), s)
    fport = np.where(has, aport, pp[sel]).astype(np.int64)          # flows the policy allows
    fproto = np.where(has, aproto, pr[sel]).astype(np.uint8)
    eport = s.randint(F, 1024, 65536)
    ing = s.frac(F) < 0.75
    d = np.where(ing[:, None], rem, loc)
    sa = np.where(ing[:, None], loc, rem)
    keys = ct6_keys(d, sa, fport, eport, fproto, np.where(ing, 1, 0))
    tcp = fproto == TCP
    seclabel = np.array([e["seclabel"] for e in eps], np.uint32)
    vals = ct_entries(F, now0, ing, tcp, np.where(ing, 0x300, seclabel[epi]), seen_non_syn=tcp, length=90)
    rk = ct6_keys(d, sa, np.zeros(F), np.zeros(F), np.full(F, ICMPV6), np.where(ing, 3, 2))
    rv = vals.copy()
    rv[:, 36] |= 0x10
    all_k = np.concatenate([keys, rk])
    uniq, first = np.unique(all_k, axis=0, return_index=True)       # twins of one pair: keep one
    cap = ct_max or max(1 << 16, 1 << int(np.ceil(np.log2(len(uniq) * 1.25 + n_pkts * v6_frac * 2 + 1))))
    maps["ct6"] = MapSpec("cilium_ct6_global", MAP_LRU_HASH, 40, 56, cap, all_k[np.sort(first)],
                          np.concatenate([vals, rv])[np.sort(first)])
    # packets: which become IPv6, of which kind (forward / reply / new / odd cases)
    v6 = s.frac(n_pkts) < v6_frac
    i6 = np.nonzero(v6)[0]
    m = len(i6)
    if not m:
        return v6
    k = kind4[i6]
    fi = np.nonzero(ing)[0][s.choice(m, max(int(ing.sum()), 1))] if ing.any() else s.choice(m, F)
    fe = np.nonzero(~ing)[0][s.choice(m, max(int((~ing).sum()), 1))] if (~ing).any() else fi
    f = np.where(k == 0, fi, fe)
    src = rem[f].copy()
    dst = loc[f].copy()
    sport = np.where(k == 0, eport[f], fport[f])
    dport = np.where(k == 0, fport[f], eport[f])
    proto = fproto[f].copy()
    new = k == 2
    nn = int(new.sum())
    nri = s.choice(nn, n_r6)
    src[new] = remote6[nri]
    dst[new] = ep_ip6[s.choice(nn, n_ep)]
    sport[new] = s.randint(nn, 1024, 65536)
    nsel = s.choice(nn, len(pp))
    nid = r_id[nri]
    nport, nproto, nhas = _allowed_l4(pol, nid, s)
    r2 = s.frac(nn)                                     # 70% to a port the policy allows
    allow = nhas & (r2 < 0.7)
    dport[new] = np.where(allow, nport, np.where(r2 < 0.85, pp[nsel], s.randint(nn, 1, 65536)))
    proto[new] = np.where(allow, nproto, pr[nsel])
    rf = s.frac(m)
    tflags = np.where(rf < 0.90, TCP_ACK, np.where(rf < 0.95, TCP_SYN, np.where(rf < 0.98, TCP_FIN | TCP_ACK, TCP_RST)))
    hop = np.full(m, 64)
    odd = s.frac(m)
    icmp_t = np.where(s.frac(m) < 0.5, 128, 129)
    proto = np.where(odd < 0.04, ICMPV6, proto).astype(np.uint8)                 # ICMPv6 echo / reply
    ns = (odd >= 0.04) & (odd < 0.045)
    proto[ns] = ICMPV6
    icmp_t[ns] = 135                                                              # neighbour solicitation
    to_rtr = (odd >= 0.045) & (odd < 0.05)
    proto[to_rtr] = ICMPV6
    icmp_t[to_rtr] = 128
    dst[to_rtr] = np.frombuffer(ROUTER_IP6, np.uint8)                             # echo to the router
    hop[(odd >= 0.05) & (odd < 0.055)] = 1
    hbh = (odd >= 0.055) & (odd < 0.08)
    world = (odd >= 0.08) & (odd < 0.10)                                          # not local: to the stack
    dst[world, 0:2] = [0x20, 0x01]
    frames[i6, :] = 0
    full = ipv6_frames(src, dst, proto, sport, dport, tflags, hop, np.broadcast_to(NODE_MAC, (m, 6)),
                       np.array([0x02, 0, 0, 0, 0, 1], np.uint8)[None].repeat(m, 0), icmp_type=icmp_t, hbh=hbh,
                       stride=max(128, frames.shape[1]))
    frames[i6] = full[:, :frames.shape[1]]                                        # (64-B records: truncated)
    nh_odd = (odd >= 0.10) & (odd < 0.105)                                        # fragment / no-next-header
    frames[i6[nh_odd], 20] = np.where(s.frac(int(nh_odd.sum())) < 0.5, 44, 59)
    ln = np.full(m, 90, np.uint32)
    short = (odd >= 0.105) & (odd < 0.11)
    ln[short] = s.randint(int(short.sum()), 14, 70).astype(np.uint32)
    ln[short & (proto == ICMPV6)] = 54                                            # icmp6_load_type past the end
    length[i6] = ln
    return v6


# --------------------------------------------------------------------------
# Config 5: from-container egress, dual stack, lb4/lb6 services (50k) + policy
# --------------------------------------------------------------------------

NODE_MAC = np.array([0xDE, 0xAD, 0xBE, 0xEF, 0xC0, 0xDE], np.uint8)     # bpf/node_config.h:51
IPV4_LOOPBACK = 0x0AF5FF1F            # 10.245.255.31 (node_config.h:45 raw 0x1ffff50a)
CLUSTER_V4 = (0x0A000000, 0xFF000000)  # IPV4_CLUSTER_RANGE / _MASK: 10.0.0.0/8
V6_POD_PREFIX = bytes([0xFD, 0, 0, 0, 0, 0, 0, 0])          # ROUTER_IP's /64 (ipv6_match_prefix_64)
ROUTER_IP6 = V6_POD_PREFIX + bytes([0, 0, 0, 0, 0, 0, 0, 1])
ICMPV6 = 58


def v6_addrs(prefix8: bytes, hi: np.ndarray, lo: np.ndarray) -> np.ndarray:
    """(n, 16) addresses: 8-byte prefix + be32 hi + be32 lo."""
    n = len(lo)
    a = np.zeros((n, 16), np.uint8)
    a[:, 0:8] = np.frombuffer(prefix8, np.uint8)
    a[:, 8:12] = be32_bytes(np.asarray(hi, np.uint32))
    a[:, 12:16] = be32_bytes(np.asarray(lo, np.uint32))
    return a


def endpoint_keys_v6(ip6: np.ndarray) -> np.ndarray:
    k = np.zeros((len(ip6), 20), np.uint8)
    k[:, 0:16] = ip6
    k[:, 16] = 2
    return k


def ipcache_keys_v6(addr6: np.ndarray, plen: np.ndarray) -> np.ndarray:
    k = np.zeros((len(addr6), 24), np.uint8)
    k[:, 0:4] = le32_bytes(np.asarray(plen, np.uint32) + 32)
    k[:, 7] = 2
    k[:, 8:24] = addr6
    return k


def lb4_keys(addr, dport, slave) -> np.ndarray:
    """struct lb4_key (common.h:427-431): be32 address, be16 dport, u16 slave."""
    n = len(addr)
    k = np.zeros((n, 8), np.uint8)
    k[:, 0:4] = be32_bytes(np.asarray(addr, np.uint32))
    k[:, 4:6] = be16_bytes(np.asarray(dport, np.uint16))
    k[:, 6:8] = le16_bytes(np.asarray(slave, np.uint16))
    return k


def lb4_services(target, port, count, rev_nat, weight) -> np.ndarray:
    """struct lb4_service (common.h:433-439) as pkg/maps/lbmap writes it: port, rev_nat
    and weight in network order (Service4Value.ToNetwork), count host order."""
    n = len(target)
    v = np.zeros((n, 12), np.uint8)
    v[:, 0:4] = be32_bytes(np.asarray(target, np.uint32))
    v[:, 4:6] = be16_bytes(np.asarray(port, np.uint16))
    v[:, 6:8] = le16_bytes(np.asarray(count, np.uint16))
    v[:, 8:10] = be16_bytes(np.asarray(rev_nat, np.uint16))
    v[:, 10:12] = be16_bytes(np.asarray(weight, np.uint16))
    return v


def lb6_keys(addr6, dport, slave) -> np.ndarray:
    n = len(addr6)
    k = np.zeros((n, 20), np.uint8)
    k[:, 0:16] = addr6
    k[:, 16:18] = be16_bytes(np.asarray(dport, np.uint16))
    k[:, 18:20] = le16_bytes(np.asarray(slave, np.uint16))
    return k


def lb6_services(target6, port, count, rev_nat, weight) -> np.ndarray:
    n = len(target6)
    v = np.zeros((n, 24), np.uint8)
    v[:, 0:16] = target6
    v[:, 16:18] = be16_bytes(np.asarray(port, np.uint16))
    v[:, 18:20] = le16_bytes(np.asarray(count, np.uint16))
    v[:, 20:22] = be16_bytes(np.asarray(rev_nat, np.uint16))
    v[:, 22:24] = be16_bytes(np.asarray(weight, np.uint16))
    return v


def revnat4(index, addr, port):
    """cilium_lb4_reverse_nat: be16 index -> {be32 address, be16 port} (lbmap RevNat4*.ToNetwork)."""
    k = be16_bytes(np.asarray(index, np.uint16)).copy()
    v = np.zeros((len(addr), 6), np.uint8)
    v[:, 0:4] = be32_bytes(np.asarray(addr, np.uint32))
    v[:, 4:6] = be16_bytes(np.asarray(port, np.uint16))
    return k, v


def revnat6(index, addr6, port):
    k = be16_bytes(np.asarray(index, np.uint16)).copy()
    v = np.zeros((len(addr6), 18), np.uint8)
    v[:, 0:16] = addr6
    v[:, 16:18] = be16_bytes(np.asarray(port, np.uint16))
    return k, v


def ipv6_frames(saddr6, daddr6, proto, sport, dport, tcp_flags, hoplimit, smac, dmac,
                icmp_type=None, hbh=None, stride: int = 128) -> np.ndarray:
    """Ethernet + IPv6 (+ optional 8-B hop-by-hop header) + L4 records."""
    n = len(saddr6)
    f = np.zeros((n, stride), np.uint8)
    f[:, 0:6] = dmac
    f[:, 6:12] = smac
    f[:, 12:14] = be16_bytes(np.full(n, ETH_P_IPV6, np.uint16))
    f[:, 14] = 0x60
    f[:, 18:20] = be16_bytes(np.full(n, 40, np.uint16))
    proto = np.asarray(proto, np.uint8)
    hbh = np.zeros(n, bool) if hbh is None else np.asarray(hbh, bool)
    f[:, 20] = np.where(hbh, 0, proto)
    f[:, 21] = np.asarray(hoplimit, np.uint8)
    f[:, 22:38] = saddr6
    f[:, 38:54] = daddr6
    f[hbh, 54] = proto[hbh]                          # hop-by-hop: nexthdr, hdrlen 0 (8 bytes)
    l4 = np.where(hbh, 62, 54)
    rows = np.arange(n)
    sp = be16_bytes(np.asarray(sport, np.uint16))
    dp = be16_bytes(np.asarray(dport, np.uint16))
    ports = (proto == TCP) | (proto == UDP)
    for j in range(2):
        f[rows[ports], l4[ports] + j] = sp[ports, j]
        f[rows[ports], l4[ports] + 2 + j] = dp[ports, j]
    tcp = proto == TCP
    f[rows[tcp], l4[tcp] + 12] = 0x50
    f[rows[tcp], l4[tcp] + 13] = np.asarray(tcp_flags, np.uint8)[tcp]
    if icmp_type is not None:
        ic = proto == ICMPV6
        f[rows[ic], l4[ic]] = np.asarray(icmp_type, np.uint8)[ic]
    return f


def flow_hash32(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """A per-flow stand-in for the kernel's skb hash (get_hash_recalc): the same
    5-tuple always hashes the same (the kernel's key is boot-random, so the hash is
    an input of the verdict, not an output to match)."""
    with np.errstate(over="ignore"):
        z = (a.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ (b.astype(np.uint64) << np.uint64(17)) \
            ^ c.astype(np.uint64)
        z = (z ^ (z >> np.uint64(31))) * np.uint64(0xBF58476D1CE4E5B9)
        z = z ^ (z >> np.uint64(29))
    return (z >> np.uint64(16)).astype(np.uint32)


def per_endpoint_ct(w: Workload, max_entries: int, family: str = "ct4") -> List[MapSpec]:
    """ConntrackLocal (pkg/endpoint/bpf.go:182-187, bpf_lxc.c:53-75): every endpoint its own
    CT map of `max_entries` (ctmap.go:54: 64000 per endpoint) holding the preloaded entries
    of its own flows -- the global map's entries whose address is the endpoint's, the first
    max_entries of them in insertion order (an agent never holds more)."""
    spec = w.maps[family]
    alen = 4 if family == "ct4" else 16
    if alen == 4:
        ips = np.array([e["ip"] for e in w.endpoints], np.uint32)
        da = spec.keys[:, 0:4].copy().view(">u4").reshape(-1).astype(np.uint32)
        sa = spec.keys[:, 4:8].copy().view(">u4").reshape(-1).astype(np.uint32)
        order = np.argsort(ips)
        def owner(a):
            pos = np.clip(np.searchsorted(ips[order], a), 0, len(ips) - 1)
            return np.where(ips[order][pos] == a, order[pos], -1)
        ep = owner(da)
        ep = np.where(ep >= 0, ep, owner(sa))
    else:
        where = {bytes(e["ip6"]): i for i, e in enumerate(w.endpoints)}
        ep = np.array([where.get(bytes(k[0:16]), where.get(bytes(k[16:32]), -1)) for k in spec.keys], np.int64)
    out = []
    order = np.argsort(ep, kind="stable")                          # (insertion order within an endpoint)
    bounds = np.searchsorted(ep[order], np.arange(len(w.endpoints) + 1))
    for i in range(len(w.endpoints)):
        idx = order[bounds[i]:bounds[i + 1]][:max_entries]
        out.append(MapSpec(f"cilium_{family}_{w.endpoints[i]['lxc_id']:05d}", spec.type, spec.key_size, spec.val_size,
                           max_entries, spec.keys[idx], spec.vals[idx]))
    return out


def config5(n_pkts: int = 1 << 20, seed: int = 0xC1A00005, n_svc: int = 50000, n_ep: int = 4096,
            n_remote: int = 16384, v6_frac: float = 0.5, vip_frac: float = 0.70, reply_frac: float = 0.20,
            n_flows: Optional[int] = None, ct_max: Optional[int] = None, stride: Optional[int] = None,
            family: Optional[int] = None, odd_frac: float = 1.0, ep_zipf: Optional[float] = None) -> Workload:
    """Egress from local pods through lb4/lb6 services, dual stack.

    Tables: 4096 local endpoints (v4 10.0.x.y + v6 fd00::a:x, each its own MAC),
    16k remote pods (ipcache only), 50k services (half v4, half v6; half L4, half
    L3) with 1-16 backends drawn from local + remote pods, rev-NAT entries, one
    policy map with ingress and egress L4/L3 rules, empty v4/v6 conntrack.
    Packets: `vip_frac` to service VIPs, the rest pod-to-pod / to the world,
    `reply_frac` of the pod-to-pod / service flows sent back by their responder;
    TCP/UDP/ICMP(v6) mix, with rare invalid MACs / source IPs / TTL 1 / ARP /
    unknown protocols / hop-by-hop headers.  `family` 4 or 6 restricts the batch.
    """
    s = Stream(seed)
    stride = stride or (64 if family == 4 else 128)
    n_flows = n_flows or max(n_pkts // 4, 1)
    ep_idx = np.arange(n_ep)
    ep_ip4 = np.uint32(0x0A000000) | (ep_idx + 256).astype(np.uint32)                 # 10.0.1.0 ...
    ep_ip6 = v6_addrs(V6_POD_PREFIX, np.full(n_ep, 0x000A0000), (ep_idx + 0x100).astype(np.uint32) * 0x10001)
    ep_mac = np.zeros((n_ep, 6), np.uint8)
    ep_mac[:, 0] = 0x02
    ep_mac[:, 4:6] = be16_bytes((ep_idx + 1).astype(np.uint16))
    seclabel = (0x2000 + ep_idx).astype(np.uint32)
    remote4 = (np.uint32(0x0A100000) | np.arange(n_remote, dtype=np.uint32))          # 10.16.0.0/16-ish
    remote6 = v6_addrs(V6_POD_PREFIX, np.full(n_remote, 0x00100000), np.arange(n_remote, dtype=np.uint32) + 1)
    remote_id = (0x3000 + s.choice(n_remote, 4000)).astype(np.uint32)

    # cilium_lxc: local endpoints v4 + v6, plus 2 host addresses
    host4 = np.array([0x0A0000FE, 0x0A0000FD], np.uint32)
    lk = np.concatenate([endpoint_keys_v4(ep_ip4), endpoint_keys_v6(ep_ip6), endpoint_keys_v4(host4)])
    lv = np.concatenate([endpoint_infos(100 + ep_idx, ep_idx + 1, np.zeros(n_ep)),
                         endpoint_infos(100 + ep_idx, ep_idx + 1, np.zeros(n_ep)),
                         endpoint_infos([0, 0], [0, 0], [1, 1])])
    lv[:2 * n_ep, 16:22] = np.concatenate([ep_mac, ep_mac])
    maps = {"lxc": MapSpec("cilium_lxc", MAP_HASH, 20, 48, 65536, lk, lv)}

    # ipcache: every pod /32 (/128), a few CIDRs, world
    cid4 = s.u32(512) & prefix_mask(np.full(512, 16))
    ik = np.concatenate([ipcache_keys_v4(ep_ip4, np.full(n_ep, 32)), ipcache_keys_v4(remote4, np.full(n_remote, 32)),
                         ipcache_keys_v4(cid4, np.full(512, 16)), ipcache_keys_v4(np.zeros(1, np.uint32), np.zeros(1)),
                         ipcache_keys_v6(ep_ip6, np.full(n_ep, 128)), ipcache_keys_v6(remote6, np.full(n_remote, 128))])
    ids4 = np.concatenate([seclabel, remote_id, (0x4000 + s.choice(512, 64)).astype(np.uint32),
                           np.full(1, WORLD_ID, np.uint32), seclabel, remote_id])
    maps["ipcache"] = MapSpec("cilium_ipcache", MAP_LPM_TRIE, 24, 8, 512000, ik, remote_endpoint_infos(ids4))

    # services: half v4, half v6; half L4 (port), half L3 (port 0); 1..16 backends
    n4 = n_svc // 2
    n6 = n_svc - n4
    rev = np.arange(1, n_svc + 1, dtype=np.uint32)
    fam_pods4 = np.concatenate([ep_ip4, remote4])
    fam_pods6 = np.concatenate([ep_ip6, remote6])
    svc_l4 = s.frac(n_svc) < 0.5
    svc_port = np.where(svc_l4, np.array([80, 443, 8080, 53, 9090], np.int64)[s.choice(n_svc, 5)], 0)
    nbe = s.randint(n_svc, 1, 17)
    be_port = np.where(s.frac(n_svc) < 0.5, svc_port, s.randint(n_svc, 1024, 32768))
    vip4 = (np.uint32(0xAC140000) | np.arange(n4, dtype=np.uint32))                   # 172.20.0.0/16
    vip6 = v6_addrs(bytes([0xFD, 0, 0, 0, 0, 0, 0xFF, 0xFF]), np.zeros(n6), np.arange(n6, dtype=np.uint32))
    tot_be = int(nbe.sum())
    be_pick = s.choice(tot_be, n_ep + n_remote)
    svc_of_be = np.repeat(np.arange(n_svc), nbe)
    slave_of_be = np.arange(tot_be) - np.repeat(np.cumsum(nbe) - nbe, nbe) + 1
    be4 = svc_of_be < n4
    k4 = np.concatenate([lb4_keys(vip4, svc_port[:n4], np.zeros(n4)),
                         lb4_keys(vip4[svc_of_be[be4]], svc_port[svc_of_be[be4]], slave_of_be[be4])])
    v4 = np.concatenate([lb4_services(np.zeros(n4), np.zeros(n4), nbe[:n4], np.zeros(n4), np.zeros(n4)),
                         lb4_services(fam_pods4[be_pick[be4]], be_port[svc_of_be[be4]], np.zeros(int(be4.sum())),
                                      rev[svc_of_be[be4]], np.zeros(int(be4.sum())))])
    i6 = svc_of_be[~be4] - n4
    k6 = np.concatenate([lb6_keys(vip6, svc_port[n4:], np.zeros(n6)),
                         lb6_keys(vip6[i6], svc_port[svc_of_be[~be4]], slave_of_be[~be4])])
    v6 = np.concatenate([lb6_services(np.zeros((n6, 16), np.uint8), np.zeros(n6), nbe[n4:], np.zeros(n6), np.zeros(n6)),
                         lb6_services(fam_pods6[be_pick[~be4]], be_port[svc_of_be[~be4]], np.zeros(int((~be4).sum())),
                                      rev[svc_of_be[~be4]], np.zeros(int((~be4).sum())))])
    cap_lb = 1 << int(np.ceil(np.log2(max(len(k4), len(k6)) * 1.25)))
    maps["lb4_services"] = MapSpec("cilium_lb4_services", MAP_HASH, 8, 12, cap_lb, k4, v4)
    maps["lb6_services"] = MapSpec("cilium_lb6_services", MAP_HASH, 20, 24, cap_lb, k6, v6)
    rk4, rv4 = revnat4(rev[:n4], vip4, svc_port[:n4])
    rk6, rv6 = revnat6(rev[n4:], vip6, svc_port[n4:])
    maps["lb4_revnat"] = MapSpec("cilium_lb4_reverse_nat", MAP_HASH, 2, 6, 65536, rk4, rv4)
    maps["lb6_revnat"] = MapSpec("cilium_lb6_reverse_nat", MAP_HASH, 2, 18, 65536, rk6, rv6)

    # policy (one map for every endpoint): pod identities x {80,443,8080,53,9090,
    # backend ports} egress + ingress, L3 allow for 20% of identities, wildcards
    all_ids = np.unique(np.concatenate([seclabel, remote_id]))
    ports = np.array([80, 443, 8080, 53, 9090], np.int64)
    pk = []
    for eg in (0, 1):
        rid = np.repeat(all_ids, len(ports) * 2)
        rp = np.tile(np.repeat(ports, 2), len(all_ids))
        rpr = np.tile([TCP, UDP], len(all_ids) * len(ports))
        keep = s.frac(len(rid)) < 0.7
        pk.append(policy_keys(rid[keep], rp[keep], rpr[keep], eg))
        l3 = np.concatenate([all_ids[s.frac(len(all_ids)) < 0.4], [WORLD_ID] if eg else []]).astype(np.uint32)
        pk.append(policy_keys(l3, np.zeros(len(l3)), np.zeros(len(l3)), eg))
        wp = s.randint(32, 1024, 32768)
        pk.append(policy_keys(np.zeros(32), wp, np.full(32, TCP), eg))
    pk = np.unique(np.concatenate(pk), axis=0)
    proxy = np.where(s.frac(len(pk)) < 0.02, s.randint(len(pk), 10000, 20000), 0)
    maps["policy"] = MapSpec("cilium_policy", MAP_HASH, 8, 24, 1 << int(np.ceil(np.log2(len(pk) * 1.25))),
                             pk, policy_entries(proxy))
    cap = ct_max or max(1 << 16, 1 << int(np.ceil(np.log2(n_flows * 8))))
    maps["ct4"] = MapSpec("cilium_ct4_global", MAP_LRU_HASH, 14, 56, cap, np.zeros((0, 14), np.uint8),
                          np.zeros((0, 56), np.uint8))
    maps["ct6"] = MapSpec("cilium_ct6_global", MAP_LRU_HASH, 40, 56, cap, np.zeros((0, 40), np.uint8),
                          np.zeros((0, 56), np.uint8))

    # ---- flows: (family, client ep, destination kind, dst, ports, proto)
    F = n_flows
    fam6 = (s.frac(F) < v6_frac) if family is None else np.full(F, family == 6)
    cli = s.choice(F, n_ep)
    if ep_zipf:                                                    # (the busiest clients: Zipf(a) over endpoints)
        cli = zipf_ranks(Stream(seed ^ 0xE9E9E9E9), F, n_ep, ep_zipf)
    r = s.frac(F)
    kind = np.where(r < vip_frac, 0, np.where(r < vip_frac + 0.15, 1, np.where(r < vip_frac + 0.25, 2, 3)))
    # 0 service, 1 local pod, 2 remote pod, 3 world
    svc = np.where(fam6, n4 + s.choice(F, n6), s.choice(F, n4))
    rp = s.frac(F)
    proto = np.where(rp < 0.80, TCP, np.where(rp < 0.95, UDP, ICMP)).astype(np.uint8)
    proto = np.where(fam6 & (proto == ICMP), ICMPV6, proto).astype(np.uint8)
    sport = s.randint(F, 1024, 65536)
    dport = np.where(kind == 0, np.where(svc_port[svc] > 0, svc_port[svc], ports[s.choice(F, 5)]),
                     ports[s.choice(F, 5)])
    dst_ep = s.choice(F, n_ep)
    dst_rm = s.choice(F, n_remote)
    world4 = (np.uint32(0x08000000) | s.u32(F) >> np.uint32(8))
    d4 = np.where(kind == 0, vip4[np.minimum(svc, n4 - 1)],
                  np.where(kind == 1, ep_ip4[dst_ep], np.where(kind == 2, remote4[dst_rm], world4)))
    d6 = np.where((kind == 0)[:, None], vip6[np.clip(svc - n4, 0, n6 - 1)],
                  np.where((kind == 1)[:, None], ep_ip6[dst_ep],
                           np.where((kind == 2)[:, None], remote6[dst_rm],
                                    v6_addrs(bytes([0x20, 0x01, 0x0D, 0xB8, 0, 0, 0, 0]), s.u32(F), s.u32(F)))))
    fh = flow_hash32(cli.astype(np.uint64) * 65536 + sport, np.where(fam6, svc, d4.astype(np.int64)), dport)
    # the responder of a flow: the destination pod, or the service backend the
    # flow's hash selects (lb_select_slave: hash % count + 1)
    slave = (fh % nbe[svc].astype(np.uint32)).astype(np.int64) + 1
    be_base = np.cumsum(nbe) - nbe
    be_row = be_base[svc] + slave - 1
    resp4 = np.where(kind == 0, fam_pods4[be_pick[be_row]], d4)
    resp6 = np.where((kind == 0)[:, None], fam_pods6[be_pick[be_row]], d6)
    resp_port = np.where((kind == 0) & (be_port[svc] > 0), be_port[svc], dport)
    # responder endpoint index if local (replies are only generated from local pods)
    off4 = resp4.astype(np.int64) - int(ep_ip4[0])                 # ep_ip4 is contiguous
    resp_ep = np.where((off4 >= 0) & (off4 < n_ep), off4, -1)
    if kind.size:
        is_loc6 = (resp6[:, 8:12].view(">u4").reshape(-1) == 0x000A0000) & (resp6[:, :8] == np.frombuffer(V6_POD_PREFIX, np.uint8)).all(1)
        lo6 = resp6[:, 12:16].view(">u4").reshape(-1).astype(np.int64) // 0x10001 - 0x100
        resp_ep6 = np.where(is_loc6 & (lo6 >= 0) & (lo6 < n_ep), lo6, -1)
        resp_ep = np.where(fam6, resp_ep6, resp_ep)

    # ---- packets
    fi = s.choice(n_pkts, F)
    rep = (s.frac(n_pkts) < reply_frac) & (resp_ep[fi] >= 0) & (kind[fi] <= 1)
    f6 = fam6[fi]
    src_ep = np.where(rep, resp_ep[fi], cli[fi]).astype(np.uint16)
    rf = s.frac(n_pkts)
    tflags = np.where(rf < 0.90, TCP_ACK, np.where(rf < 0.95, TCP_SYN, np.where(rf < 0.98, TCP_FIN | TCP_ACK, TCP_RST)))
    pr = proto[fi]
    p_sport = np.where(rep, resp_port[fi], sport[fi])
    p_dport = np.where(rep, sport[fi], dport[fi])
    icmp_t = np.where(rep, np.where(f6, 129, 0), np.where(f6, 128, 8))
    ttl = np.full(n_pkts, 64)
    smac = ep_mac[src_ep]
    dmac = np.broadcast_to(NODE_MAC, (n_pkts, 6)).copy()
    # rare odd cases
    odd = s.frac(n_pkts)
    o = odd_frac
    smac[odd < 0.001 * o] = 0x33
    dmac[(odd >= 0.001 * o) & (odd < 0.002 * o)] = 0x44
    ttl[(odd >= 0.002 * o) & (odd < 0.0025 * o)] = 1
    pr = np.where((odd >= 0.0025 * o) & (odd < 0.0035 * o), 47, pr).astype(np.uint8)     # GRE: unknown L4
    bad_sip = (odd >= 0.0035 * o) & (odd < 0.0045 * o)
    hbh = f6 & (odd >= 0.0045 * o) & (odd < 0.0145 * o)
    arp = (odd >= 0.0145 * o) & (odd < 0.0155 * o)
    ns6 = f6 & (odd >= 0.0155 * o) & (odd < 0.0160 * o)
    frames = np.zeros((n_pkts, stride), np.uint8)
    i4 = np.nonzero(~f6)[0]
    if len(i4):
        sa = np.where(rep[i4], resp4[fi[i4]], ep_ip4[src_ep[i4]]).astype(np.uint32)
        da = np.where(rep[i4], ep_ip4[cli[fi[i4]]], d4[fi[i4]]).astype(np.uint32)
        sa = np.where(bad_sip[i4], sa ^ np.uint32(0x00000F00), sa).astype(np.uint32)
        fr = ipv4_frames(sa, da, pr[i4], p_sport[i4], p_dport[i4], tflags[i4], ttl[i4],
                         np.where(arp[i4], ETH_P_ARP, ETH_P_IP), stride=stride, icmp_type=icmp_t[i4])
        fr[:, 0:6] = dmac[i4]
        fr[:, 6:12] = smac[i4]
        frames[i4] = fr
    i6 = np.nonzero(f6)[0]
    if len(i6):
        if stride < 128:
            raise ValueError("IPv6 records need stride 128")
        sa6 = np.where(rep[i6][:, None], resp6[fi[i6]], ep_ip6[src_ep[i6]])
        da6 = np.where(rep[i6][:, None], ep_ip6[cli[fi[i6]]], d6[fi[i6]])
        sa6 = sa6.copy()
        sa6[bad_sip[i6], 15] ^= 0x5A
        pr6 = pr[i6].copy()
        it6 = icmp_t[i6].copy()
        pr6[ns6[i6]] = ICMPV6
        it6[ns6[i6]] = 135
        frames[i6] = ipv6_frames(sa6, da6, pr6, p_sport[i6], p_dport[i6], tflags[i6], ttl[i6], smac[i6], dmac[i6],
                                 icmp_type=it6, hbh=hbh[i6], stride=stride)
    fhash = np.where(rep, flow_hash32(fh[fi].astype(np.uint64), np.full(n_pkts, 7), p_dport), fh[fi]).astype(np.uint32)
    length = np.where(f6, 90, 64).astype(np.uint32)
    eps = [{"lxc_id": int(i + 1), "seclabel": int(seclabel[i]), "ip": int(ep_ip4[i]), "ip6": bytes(ep_ip6[i]),
            "mac": bytes(ep_mac[i]), "node_mac": bytes(NODE_MAC), "ifindex": int(100 + i)} for i in range(n_ep)]
    return Workload("config5", maps, frames, length, np.zeros(n_pkts, np.uint32), eps, now=2_000_000,
                    extra={"src_ep": src_ep, "flow_hash": fhash,
                           "node": {"cluster_mask": CLUSTER_V4[1], "cluster_range": CLUSTER_V4[0],
                                    "loopback": IPV4_LOOPBACK, "router_ip6": ROUTER_IP6,
                                    "host_mac": bytes([0x02, 0x00, 0x00, 0x00, 0xFE, 0x01])},
                           "kind": kind[fi], "reply": rep, "v6": f6, "flow": fi, "hbh": hbh})


# --------------------------------------------------------------------------
# Benchmark steps of the stateful configs
# --------------------------------------------------------------------------

def port_variant(w: Workload, v: int, fresh_frac: float = 0.2):
    """Step v (>= 1) of a stateful benchmark: the batch with fresh client ports on its
    new flows, so every step creates conntrack entries the way the workload says
    instead of replaying flows an earlier step created.  Config 3 / 4: every new-flow
    packet (kind 2) takes source port 1024 + (sport - 1024 + 4099 v) mod 64512.
    Config 5: the flows whose (flow, v) hash falls under fresh_frac take that client
    port (the source port of the client's packets, the destination port of the
    replies); the other flows keep theirs and stay established.  v = 0 is the batch
    itself.  Returns (rows, byte offsets of the 2-byte port, new port values)."""
    f = w.frames
    key = ("_pv", fresh_frac if w.name == "config5" else None)
    if w.name == "config3" and key in (w.extra or {}):
        rows, offs, old = w.extra[key]                # (the new-flow rows do not depend on v)
        rows, offs = (rows[:0], offs[:0]) if v == 0 else (rows, offs)
        return rows, offs, 1024 + (old[:len(rows)] - 1024 + 4099 * v) % 64512
    if w.name == "config3":
        rows = np.nonzero(w.extra["kind"] == 2)[0]
        v6 = w.extra.get("v6")
        if v6 is not None:
            rows = rows[~v6[rows]]
        proto = f[rows, 23]
        rows = rows[(proto == TCP) | (proto == UDP)]
        offs = 14 + 4 * (f[rows, 14] & 0xF).astype(np.int64)
    elif w.name == "config5":
        fl = w.extra["flow"].astype(np.uint64)
        with np.errstate(over="ignore"):
            h = splitmix64(0x5EED0000 + v, 1)[0] ^ (fl * GOLDEN)
        h = (h ^ (h >> np.uint64(31))) * np.uint64(0xBF58476D1CE4E5B9)
        fresh = ((h >> np.uint64(40)).astype(np.float64) / float(1 << 24)) < fresh_frac
        v6 = w.extra["v6"]
        l4 = np.where(v6, np.where(w.extra["hbh"], 62, 54), 34)
        nh6 = f[:, 54] if f.shape[1] > 54 else np.zeros(w.n, np.uint8)
        proto = np.where(v6, np.where(w.extra["hbh"], nh6, f[:, 20]), f[:, 23])
        ok = fresh & ((proto == TCP) | (proto == UDP)) & (l4 + 4 <= f.shape[1])
        rows = np.nonzero(ok)[0]
        offs = l4[rows] + np.where(w.extra["reply"][rows], 2, 0)
    else:
        raise ValueError(w.name)
    old = (f[rows, offs].astype(np.int64) << 8) | f[rows, offs + 1]
    if w.name == "config3" and w.extra is not None:
        w.extra[key] = (rows, offs, old)
    if v == 0:
        rows, offs, old = rows[:0], offs[:0], old[:0]
    new = 1024 + (old - 1024 + 4099 * v) % 64512
    return rows, offs, new.astype(np.int64)
