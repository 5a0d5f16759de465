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
from typing import Dict, List, Optional

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


def config3(n_pkts: int = 1 << 24, n_flows: int = 1 << 24, seed: int = 0xC1A00003, now0: int = 1_000_000,
            n_cidrs: int = 102400, n_ids: int = 10000, n_ep: int = 4096, ct_max: Optional[int] = None,
            ttl_low: float = 0.0005) -> Workload:
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
    pick = s.choice(n_flows, len(cidr_addr))
    remote = _rand_addrs_in(s, cidr_addr[pick], cidr_plen[pick])
    epi = s.choice(n_flows, n_ep)
    local = lxc_ip[epi]
    pol = c2.maps["policy"].keys
    pol_port = pol[:, 4:6].copy().view(">u2").reshape(-1)
    pol_proto = pol[:, 6]
    l4 = pol_proto != 0
    pp, pr = pol_port[l4], pol_proto[l4]
    sel = s.choice(n_flows, len(pp))
    fport = pp[sel].astype(np.int64)
    fproto = pr[sel].astype(np.uint8)
    eport = s.randint(n_flows, 1024, 65536)
    ingress_init = s.frac(n_flows) < 0.75
    # CT entries: ingress-initiated {daddr remote, saddr local, dport fport, sport eport, IN}
    #             egress-initiated  {daddr local, saddr remote, dport fport(remote), sport eport(local), OUT}
    d_addr = np.where(ingress_init, remote, local)
    s_addr = np.where(ingress_init, local, remote)
    keys = ct4_keys(d_addr, s_addr, fport, eport, fproto, np.where(ingress_init, 1, 0))
    tcp = fproto == TCP
    seclabel = (0x1000 + ep_ids[epi]).astype(np.uint32)
    ident = c2.maps["ipcache"].vals[pick, 0:4].copy().view("<u4").reshape(-1)
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
    kind = np.where(r < 0.6, 0, np.where(r < 0.8, 1, 2))
    f = np.where(kind == 0, fi, fe)
    saddr = remote[f].copy()
    daddr = local[f].copy()
    sport = np.where(kind == 0, eport[f], fport[f])
    dport = np.where(kind == 0, fport[f], eport[f])
    proto = fproto[f].copy()
    new = kind == 2
    nn = int(new.sum())
    npk = s.choice(nn, len(cidr_addr))
    saddr[new] = _rand_addrs_in(s, cidr_addr[npk], cidr_plen[npk])
    daddr[new] = lxc_ip[s.choice(nn, n_ep)]
    sport[new] = s.randint(nn, 1024, 65536)
    nsel = s.choice(nn, len(pp))
    dport[new] = np.where(s.frac(nn) < 0.8, pp[nsel], s.randint(nn, 1, 65536))
    proto[new] = pr[nsel]
    rf = s.frac(n_pkts)
    flags = np.where(rf < 0.90, TCP_ACK, np.where(rf < 0.95, TCP_SYN, np.where(rf < 0.98, TCP_FIN | TCP_ACK, TCP_RST)))
    ttl = np.where(s.frac(n_pkts) < ttl_low, 1, 64)
    frames = ipv4_frames(saddr, daddr, proto, sport, dport, flags, ttl)
    eps = [{"lxc_id": int(i), "seclabel": int(0x1000 + i), "ip": int(lxc_ip[i - 1])} for i in ep_ids]
    return Workload("config3", maps, frames, np.full(n_pkts, 64, np.uint32), np.zeros(n_pkts, np.uint32), eps,
                    now=now0 + 1, extra={"kind": kind})
