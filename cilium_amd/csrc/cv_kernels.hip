// cv_kernels.hip — gfx950 kernels of the batch verdict engine.
//
// One lane = one packet.  Each kernel restates a path of the reference's BPF
// programs (Taeung/cilium v1.1.90) over a batch of frame records in HBM:
//   k_xdp_prefilter    bpf/bpf_xdp.c:88-184                      (config 1)
//   k_policy_ingress   bpf/bpf_netdev.c:128-153,357-398 +
//                      bpf/lib/policy.h:217-329                   (config 2)
//   k_netdev_front     bpf/bpf_netdev.c:357-524, bpf/lib/l3.h:247-276
//   k_ct_stage         bpf/bpf_lxc.c:865-992, bpf/lib/conntrack.h (config 3)
// Map lookups are the table probes of cv_hash.hpp / cv_lpm.hpp; counters use
// device atomics; cilium_metrics is aggregated per workgroup in LDS and flushed
// once per workgroup.  No MFMA: this is integer gather work, HBM/L2 bound.
#include <errno.h>
#include <hip/hip_runtime.h>

#include "cv_dp.hpp"

namespace cv {

constexpr int BLOCK = 256;
constexpr uint32_t NONE = 0xFFFFFFFFu;

// ------------------------------------------------------------------ records
// The first 64 bytes of a frame record live in 16 VGPRs; bytes beyond come from
// HBM (rare: IP options).  Loads use the non-temporal path so the streamed
// records do not evict the tables from L2 / Infinity Cache.
struct Rec {
    uint32_t w[16];
    const uint8_t *base;
    uint32_t len, stride;
};

__device__ __forceinline__ void rec_load(Rec &r, const BatchDev &b, uint32_t i, int nvec)
{
    r.base = b.frames + (size_t)i * b.stride;
    r.len = b.len[i];
    r.stride = b.stride;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *q = reinterpret_cast<const u32x4 *>(r.base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < nvec) {
            u32x4 v = __builtin_nontemporal_load(q + k);
            r.w[4 * k] = v.x; r.w[4 * k + 1] = v.y; r.w[4 * k + 2] = v.z; r.w[4 * k + 3] = v.w;
        } else {
            r.w[4 * k] = r.w[4 * k + 1] = r.w[4 * k + 2] = r.w[4 * k + 3] = 0;
        }
    }
}

// Fixed-offset fields come from the registers (compile-time word index); fields at
// a runtime offset (L4 behind IP options, bytes past 64) are read from HBM.
template <int O>
__device__ __forceinline__ uint32_t rec_u8c(const Rec &r)
{
    static_assert(O >= 0 && O < 64, "register window");
    return (r.w[O >> 2] >> (8 * (O & 3))) & 0xFFu;
}

template <int O>
__device__ __forceinline__ uint32_t rec_raw16c(const Rec &r)   // raw LE load of 2 network-order bytes
{
    static_assert(O >= 0 && O + 2 <= 64, "register window");
    if constexpr ((O & 3) == 3) return rec_u8c<O>(r) | (rec_u8c<O + 1>(r) << 8);
    else return (r.w[O >> 2] >> (8 * (O & 3))) & 0xFFFFu;
}

template <int O>
__device__ __forceinline__ uint32_t rec_raw32c(const Rec &r)
{
    static_assert(O >= 0 && O + 4 <= 64, "register window");
    if constexpr ((O & 3) == 0) return r.w[O >> 2];
    else return (r.w[O >> 2] >> (8 * (O & 3))) | (r.w[(O >> 2) + 1] << (32 - 8 * (O & 3)));
}

// byte K of the L4 header at runtime offset `off`: registers when off == 34 (ihl 5)
template <int K>
__device__ __forceinline__ uint32_t l4_u8(const Rec &r, int off)
{
    if (off == 34) return rec_u8c<34 + K>(r);
    return r.base[off + K];
}

template <int K>
__device__ __forceinline__ uint32_t l4_raw16(const Rec &r, int off)
{
    if (off == 34) return rec_raw16c<34 + K>(r);
    return r.base[off + K] | ((uint32_t)r.base[off + K + 1] << 8);
}

// skb_load_bytes bound: 0 ok, 1 beyond skb->len (the helper fails), E_TRUNC beyond the record
__device__ __forceinline__ int rec_chk(const Rec &r, int off, int n)
{
    if (off < 0 || (uint32_t)(off + n) > r.len) return 1;
    if ((uint32_t)(off + n) > r.stride) return E_TRUNC;
    return 0;
}

// ------------------------------------------------------------------ metrics
struct LdsMetrics {            // [256 reasons]{count, bytes}, one direction
    unsigned long long c[256 * 2];
};

__device__ __forceinline__ void lm_init(LdsMetrics &m)
{
    for (int i = threadIdx.x; i < 512; i += blockDim.x) m.c[i] = 0;
    __syncthreads();
}

__device__ __forceinline__ void lm_add(LdsMetrics &m, int32_t reason_code, uint32_t len)
{
    const uint32_t r = (uint8_t)(-reason_code);   // update_metrics(len, dir, -reason)
    atomicAdd(&m.c[2 * r], 1ull);
    atomicAdd(&m.c[2 * r + 1], (unsigned long long)len);
}

__device__ __forceinline__ void lm_flush(LdsMetrics &m, unsigned long long *g, int dir)
{
    __syncthreads();
    if (!g) return;
    for (int r = threadIdx.x; r < 256; r += blockDim.x) {
        unsigned long long c = m.c[2 * r];
        if (c) {
            atomicAdd(&g[(r * 4 + dir) * 2], c);
            atomicAdd(&g[(r * 4 + dir) * 2 + 1], m.c[2 * r + 1]);
        }
    }
}

// ------------------------------------------------------------------ lookups
struct Acct { uint32_t nl, nu; };

// lookup_ip4_endpoint (eps.h:37-46): ival = lxc_id | HOST << 16 | (ifindex != 0) << 17
__device__ __forceinline__ bool lxc4_find(const DpParams &p, uint32_t daddr_raw, uint32_t &ival, Acct &a)
{
    if (!p.lxc4.buckets) return false;
    a.nl++;
    return dev_find<LxcV4Spec>(p.lxc4, &daddr_raw, &ival) >= 0;
}

// ipcache_lookup4 (eps.h:309-319) -> remote_endpoint_info.sec_label (0 = none)
__device__ __forceinline__ uint32_t ipcache4(const DpParams &p, uint32_t saddr_raw, Acct &a)
{
    if (!p.ipc4.l1) return 0;
    a.nl++;
    return lpm4_lookup(p.ipc4, bswap32(saddr_raw));
}

// handle_identity_from_host (bpf_netdev.c:128-153)
__device__ __forceinline__ uint32_t identity_from_mark(uint32_t mark, bool &skip_proxy)
{
    const uint32_t magic = mark & 0xF00u;
    skip_proxy = false;
    if (magic == 0xA00u) { skip_proxy = true; return ((mark & 0xFFu) << 16) | (mark >> 16); }
    if (magic == 0xB00u) return ((mark & 0xFFu) << 16) | (mark >> 16);
    if (magic == 0xC00u) return HOST_ID;
    return WORLD_ID;
}

// A policy counter update held back by the lane: the atomic is issued after the
// lane's last dependent lookup, so in-order vmcnt never makes a lookup wait for it.
struct Hit {
    unsigned long long *p;
    unsigned long long inc;
};

__device__ __forceinline__ void hit_flush(const Hit &h)
{
    if (h.p) atomicAdd(h.p, h.inc);
}

// __policy_can_access (policy.h:217-285); cb[CB_POLICY] is 0 on these paths.  With
// `defer` the counter update is returned instead of issued.
__device__ __forceinline__ int policy_access(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t identity,
                                             uint32_t dport_raw, uint32_t proto, int dir, Acct &a,
                                             Hit *defer = nullptr)
{
    if (flags & F_DROP_ALL) return DROP_POLICY;
    const uint32_t eg = dir ? 0u : 1u;
    uint32_t k[2];
    int64_t s = -1;
    uint32_t px[1] = {0};
    bool l4 = false;
    if (flags & F_HAVE_L4_POLICY) {
        k[0] = identity; k[1] = (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24);
        a.nl++;
        s = dev_find<PolicySpec>(pol, k, px);
        l4 = s >= 0;
    }
    if (s < 0) {
        k[0] = identity; k[1] = eg << 24;
        a.nl++;
        s = dev_find<PolicySpec>(pol, k, px);
    }
    if (s < 0 && (flags & F_HAVE_L4_POLICY)) {
        k[0] = 0; k[1] = (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24);
        a.nl++;
        s = dev_find<PolicySpec>(pol, k, px);
        l4 = s >= 0;
    }
    if (s < 0) return DROP_POLICY;
    a.nu++;
    uint8_t *v = pol.vals + (size_t)s * pol.vstride;
    if (!(flags & (AB_NO_POLICY_ATOMICS << 16))) {
        // __sync_fetch_and_add(packets, 1) and (bytes, len) as ONE 64-bit atomic on the
        // slot's delta word {count:25 | bytes:39} (launches are chunked to <= 2^24
        // packets and folded after each chunk, so neither field can overflow)
        if (len < (1u << 15)) {
            unsigned long long *d = pol.aux + s;
            const unsigned long long inc = (1ull << 39) | len;
            if (defer) *defer = Hit{d, inc};
            else atomicAdd(d, inc);
        } else {
            atomicAdd(reinterpret_cast<unsigned long long *>(v + 8), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long *>(v + 16), (unsigned long long)len);
        }
    }
    return l4 ? (int)px[0] : TC_ACT_OK;
}

// policy_can_access_ingress (policy.h:305-329)
__device__ __forceinline__ int policy_ingress(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t src,
                                              uint32_t dport_raw, uint32_t proto, Acct &a, Hit *defer = nullptr)
{
    if (!(flags & F_POLICY_INGRESS)) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
    if (flags & F_DROP_ALL) return DROP_POLICY;
    int r = policy_access(pol, flags, len, src, dport_raw, proto, CT_INGRESS, a, defer);
    return r >= TC_ACT_OK ? r : DROP_POLICY;
}

__device__ __forceinline__ void store_out(const OutDev &o, uint32_t i, const Acct &a)
{
    if (o.nl) o.nl[i] = (uint8_t)a.nl;
    if (o.nu) o.nu[i] = (uint8_t)a.nu;
}

// ================================================================== config 1
// check_filters / check_v4 / check_v6 (bpf_xdp.c:88-178)
__device__ __forceinline__ uint8_t xdp_verdict(const DpParams &p, const Rec &r, Acct &a)
{
    if (r.len < 14) return XDP_DROP;
    const uint32_t proto = rec_raw16c<12>(r);
    if (proto == 0x0008u) {
        if (r.len < 34) return XDP_DROP;
        uint32_t saddr = rec_raw32c<26>(r), daddr = rec_raw32c<30>(r);
        if (p.cidr4_fix.buckets) {                          // CIDR4_FILTER
            if (p.cidr4_dyn.l1) {                           // CIDR4_LPM_PREFILTER
                a.nl++;
                if (lpm4_lookup(p.cidr4_dyn, bswap32(saddr))) return XDP_DROP;
            }
            a.nl++;
            if (dev_find<Cidr4Spec>(p.cidr4_fix, &saddr, nullptr) >= 0) return XDP_DROP;
        }
        uint32_t iv;
        return lxc4_find(p, daddr, iv, a) ? XDP_PASS : XDP_DROP;
    }
    if (proto == 0xDD86u) {
        if (r.len < 54) return XDP_DROP;
        uint32_t sa[4] = {rec_raw32c<22>(r), rec_raw32c<26>(r), rec_raw32c<30>(r), rec_raw32c<34>(r)};
        uint32_t da[4] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r)};
        if (p.cidr6_fix.buckets) {
            if (p.cidr6_dyn.h.buckets) {
                a.nl++;
                if (lpm6_lookup(p.cidr6_dyn, sa)) return XDP_DROP;
            }
            a.nl++;
            if (dev_find<Cidr6Spec>(p.cidr6_fix, sa, nullptr) >= 0) return XDP_DROP;
        }
        if (!p.lxc6.buckets) return XDP_DROP;
        a.nl++;
        uint32_t iv;
        return dev_find<LxcV6Spec>(p.lxc6, da, &iv) >= 0 ? XDP_PASS : XDP_DROP;
    }
    return XDP_PASS;
}

__global__ void __launch_bounds__(BLOCK) k_xdp_prefilter(DpParams p, BatchDev b, OutDev o)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        Rec r;
        rec_load(r, b, i, 4);
        Acct a{0, 0};
        const uint8_t v = xdp_verdict(p, r, a);
        if (o.xdp) o.xdp[i] = v;
        store_out(o, i, a);
    }
}

// ================================================================== config 2
// The L4 key of a NEW flow as ct_lookup4 (conntrack.h:471-530) leaves it after the
// reversed lookup: returns 0 and dport/proto, or DROP_* / E_TRUNC.
__device__ __forceinline__ int l4_key_new_flow(const Rec &r, uint32_t &dport_raw, uint32_t &proto)
{
    proto = rec_u8c<23>(r);
    const int off = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
    int c;
    switch (proto) {
    case 1:                                                      // ICMP
        c = rec_chk(r, off, 1);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        dport_raw = l4_u8<0>(r, off) == 8 ? 8u : 0u;              // ECHO: sport = type, then reversed
        return 0;
    case 6:                                                      // TCP: flags then ports
        c = rec_chk(r, off + 12, 2);
        if (!c) c = rec_chk(r, off, 4);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        dport_raw = l4_raw16<2>(r, off);
        return 0;
    case 17:                                                     // UDP
        c = rec_chk(r, off, 4);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        dport_raw = l4_raw16<2>(r, off);
        return 0;
    default:
        return DROP_CT_UNKNOWN_PROTO;
    }
}

// PPT packets per lane: lane t of workgroup w takes packets w*PPT*BLOCK + k*BLOCK + t
// (coalesced per k); its policy counter atomics wait in registers until its last
// lookup is done.
constexpr int PPT = 4;

__global__ void __launch_bounds__(BLOCK) k_policy_ingress(DpParams p, int ep, BatchDev b, OutDev o)
{
    __shared__ LdsMetrics lm;
    lm_init(lm);
    const HashTable pol = p.eps[ep].policy;
    Hit hits[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        hits[k] = Hit{nullptr, 0};
        const uint32_t i = blockIdx.x * (PPT * BLOCK) + k * BLOCK + threadIdx.x;
        if (i >= b.n) continue;
        Rec r;
        rec_load(r, b, i, 3);
        Acct a{0, 0};
        bool skip_proxy = false;
        uint32_t identity = 0;
        if (p.flags & F_FROM_HOST) identity = identity_from_mark(b.mark ? b.mark[i] : 0u, skip_proxy);
        const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
        int32_t ret;
        uint16_t proxy = 0;
        if (eth != 0x0008u) {
            ret = DROP_UNKNOWN_L3;
        } else if (r.len < 34) {
            ret = DROP_INVALID;
        } else {
            if (identity < HEALTH_ID && !(p.ablate & AB_NO_IPCACHE)) {   // bpf_netdev.c:375-398
                const uint32_t lab = ipcache4(p, rec_raw32c<26>(r), a);
                if (lab && lab != CLUSTER_ID && lab != HOST_ID) identity = lab;
            }
            uint32_t dport, proto;
            ret = l4_key_new_flow(r, dport, proto);
            if (ret == 0) {
                const int v = (p.ablate & AB_NO_POLICY)
                                  ? (int)(identity & 1)
                                  : policy_ingress(pol, p.flags | (p.ablate << 16), r.len, identity, dport, proto, a,
                                                   &hits[k]);
                if (v < 0) ret = DROP_POLICY;
                else if (skip_proxy && v > 0) ret = 0;
                else { ret = v; proxy = v > 0 ? (uint16_t)v : 0; }
            }
        }
        if (ret < 0 && ret != E_TRUNC && !(p.ablate & AB_NO_METRICS)) lm_add(lm, ret, r.len);
        if (o.ret) o.ret[i] = ret;
        if (o.identity) o.identity[i] = identity;
        if (o.proxy) o.proxy[i] = proxy;
        if (o.ct) o.ct[i] = CT_NONE;
        store_out(o, i, a);
    }
#pragma unroll
    for (int k = 0; k < PPT; ++k) hit_flush(hits[k]);
    lm_flush(lm, p.metrics, METRIC_INGRESS);
}

// ================================================================== config 3
// ---- struct ct_entry (common.h:380-406) held in 16 words
struct CtE {
    uint32_t w[16];
    __device__ uint16_t bits() const { return (uint16_t)(w[9] & 0xFFFFu); }
    __device__ void set_bits(uint16_t b) { w[9] = (w[9] & 0xFFFF0000u) | b; }
    __device__ void add64(int k, uint64_t v)
    {
        uint64_t x = ((uint64_t)w[k + 1] << 32 | w[k]) + v;
        w[k] = (uint32_t)x; w[k + 1] = (uint32_t)(x >> 32);
    }
};

__device__ __forceinline__ void ct_load(const HashTable &t, int64_t slot, CtE &e)
{
    const uint4 *q = reinterpret_cast<const uint4 *>(t.vals + (size_t)slot * t.vstride);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint4 v = q[k];
        e.w[4 * k] = v.x; e.w[4 * k + 1] = v.y; e.w[4 * k + 2] = v.z; e.w[4 * k + 3] = v.w;
    }
}

__device__ __forceinline__ void ct_store(const HashTable &t, int64_t slot, const CtE &e)
{
    uint4 *q = reinterpret_cast<uint4 *>(t.vals + (size_t)slot * t.vstride);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = make_uint4(e.w[4 * k], e.w[4 * k + 1], e.w[4 * k + 2], e.w[4 * k + 3]);
}

// __ct_update_timeout (conntrack.h:103-161)
__device__ __forceinline__ void ct_timeout_raw(CtE &e, uint32_t lifetime, int dir, uint32_t seen, uint32_t now)
{
    e.w[8] = now + lifetime;
    const int fsh = dir == CT_INGRESS ? 24 : 16;                // rx_flags_seen @43, tx_flags_seen @42
    const int li = dir == CT_INGRESS ? 13 : 12;                 // last_rx_report @52, last_tx_report @48
    const uint32_t acc = (e.w[10] >> fsh) & 0xFFu;
    seen = (seen | acc) & 0xFFu;
    if (e.w[li] + CT_REPORT_INTERVAL < now || acc != seen) {
        e.w[li] = now;
        e.w[10] = (e.w[10] & ~(0xFFu << fsh)) | (seen << fsh);
    }
}

// ct_update_timeout (conntrack.h:169-186)
__device__ __forceinline__ void ct_timeout(CtE &e, bool tcp, int dir, uint32_t seen, uint32_t now)
{
    uint32_t lifetime = CT_LIFETIME_NONTCP;
    if (tcp) {
        if (!(seen & TCPF_SYN)) e.set_bits(e.bits() | CTB_SEEN_NON_SYN);
        lifetime = (e.bits() & CTB_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    ct_timeout_raw(e, lifetime, dir, seen, now);
}

__device__ __forceinline__ bool ct_alive(const CtE &e)
{
    return !(e.bits() & CTB_RX_CLOSING) || !(e.bits() & CTB_TX_CLOSING);
}

struct Tuple4 {                 // struct ipv4_ct_tuple packed into 4 words (+2 zero bytes)
    uint32_t daddr, saddr;
    uint32_t dport, sport;      // raw be16 values
    uint32_t nexthdr, flags;
    __device__ void key(uint32_t *k) const
    {
        k[0] = daddr; k[1] = saddr; k[2] = (dport & 0xFFFFu) | (sport << 16); k[3] = nexthdr | (flags << 8);
    }
};

enum { ACTION_UNSPEC = 0, ACTION_CREATE = 1, ACTION_CLOSE = 2 };

// __ct_lookup (conntrack.h:199-263) -> CT_NEW / CT_ESTABLISHED; *slot = hit slot
__device__ __forceinline__ int ct_lookup_one(const HashTable &ct, const Tuple4 &t, int action, int dir, bool tcp,
                                             uint32_t seen, uint32_t len, uint32_t now, uint32_t flags, int64_t &slot,
                                             Acct &a)
{
    uint32_t k[4];
    t.key(k);
    a.nl++;
    slot = dev_find<Ct4Spec>(ct, k, nullptr);
    if (slot < 0) return CT_NEW;
    a.nu++;
    CtE e;
    ct_load(ct, slot, e);
    if (ct_alive(e)) ct_timeout(e, tcp, dir, seen, now);
    if (flags & F_CT_ACCOUNTING) {
        if (dir == CT_INGRESS) { e.add64(0, 1); e.add64(2, len); }
        else                   { e.add64(4, 1); e.add64(6, len); }
    }
    if (action == ACTION_CREATE) {
        if ((e.bits() & CTB_RX_CLOSING) || (e.bits() & CTB_TX_CLOSING)) {
            e.set_bits(e.bits() & ~(CTB_RX_CLOSING | CTB_TX_CLOSING));
            ct_timeout(e, tcp, dir, seen, now);
        }
    } else if (action == ACTION_CLOSE) {
        e.set_bits(e.bits() | (dir == CT_INGRESS ? CTB_RX_CLOSING : CTB_TX_CLOSING));
        if (!ct_alive(e)) ct_timeout_raw(e, CT_CLOSE_TIMEOUT, dir, seen, now);
    }
    ct_store(ct, slot, e);
    return CT_ESTABLISHED;
}

// ct_lookup4 (conntrack.h:442-562); tuple in/out
__device__ __forceinline__ int ct_lookup4(const HashTable &ct, Tuple4 &t, const Rec &r, int off, int dir, uint32_t now,
                                          uint32_t flags, int64_t &slot, Acct &a)
{
    int action = ACTION_UNSPEC, c;
    const bool tcp = t.nexthdr == 6;
    uint32_t seen = 0;
    t.flags = dir == CT_INGRESS ? TUPLE_F_OUT : dir == CT_EGRESS ? TUPLE_F_IN : TUPLE_F_SERVICE;
    switch (t.nexthdr) {
    case 1: {
        c = rec_chk(r, off, 1);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        const uint32_t type = l4_u8<0>(r, off);
        t.sport = 0; t.dport = 0;
        if (type == 3 || type == 11 || type == 12) t.flags |= TUPLE_F_RELATED;
        else if (type == 0) t.dport = 8;
        else { if (type == 8) t.sport = type; action = ACTION_CREATE; }
        break;
    }
    case 6:
        c = rec_chk(r, off + 12, 2);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        seen = l4_u8<13>(r, off);
        action = (seen & (TCPF_RST | TCPF_FIN)) ? ACTION_CLOSE : ACTION_CREATE;
        c = rec_chk(r, off, 4);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        t.dport = l4_raw16<0>(r, off); t.sport = l4_raw16<2>(r, off);
        break;
    case 17:
        c = rec_chk(r, off, 4);
        if (c) return c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
        t.dport = l4_raw16<0>(r, off); t.sport = l4_raw16<2>(r, off);
        action = ACTION_CREATE;
        break;
    default:
        return DROP_CT_UNKNOWN_PROTO;
    }
    int ret = ct_lookup_one(ct, t, action, dir, tcp, seen, r.len, now, flags, slot, a);
    if (ret != CT_NEW) return (t.flags & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
    if (dir != CT_SERVICE) {                                     // ipv4_ct_tuple_reverse
        uint32_t x = t.saddr; t.saddr = t.daddr; t.daddr = x;
        x = t.sport; t.sport = t.dport; t.dport = x;
        t.flags ^= TUPLE_F_IN;
        ret = ct_lookup_one(ct, t, action, dir, tcp, seen, r.len, now, flags, slot, a);
    }
    return ret;
}

// ct_create4 (conntrack.h:663-744) for an ingress NEW flow (ct_state: only src_sec_id)
__device__ __forceinline__ int ct_create4_ingress(const HashTable &ct, const Tuple4 &t, uint32_t len, uint32_t src,
                                                  uint32_t now)
{
    CtE e;
#pragma unroll
    for (int k = 0; k < 16; ++k) e.w[k] = 0;
    const bool tcp = t.nexthdr == 6;
    ct_timeout(e, tcp, CT_INGRESS, tcp ? TCPF_SYN : 0u, now);
    e.w[0] = 1; e.w[2] = len;                                     // rx_packets, rx_bytes
    e.w[11] = src;                                                // src_sec_id
    uint32_t k[4];
    t.key(k);
    bool created;
    int64_t s = dev_upsert<Ct4Spec>(ct, k, &created);
    if (s < 0) return DROP_CT_CREATE_FAILED;
    ct_store(ct, s, e);
    Tuple4 it = t;                                                // ICMP-RELATED entry (:727-741)
    it.nexthdr = 1; it.sport = 0; it.dport = 0; it.flags = t.flags | TUPLE_F_RELATED;
    e.set_bits(e.bits() | CTB_SEEN_NON_SYN);
    it.key(k);
    s = dev_upsert<Ct4Spec>(ct, k, &created);
    if (s < 0) return DROP_CT_CREATE_FAILED;
    ct_store(ct, s, e);
    return 0;
}

// ipv4_policy (bpf_lxc.c:865-979), LXC_NAT46 off.  Returns the program's return
// value before tail_ipv4_policy's IS_ERR mapping.
__device__ int ipv4_policy(const DpParams &p, const EpDev &ep, const Rec &r, uint32_t src_label, bool skip_proxy,
                           bool ifindex_nz, uint32_t now, uint8_t &ct_out, uint16_t &proxy, Acct &a)
{
    Tuple4 t;
    t.nexthdr = rec_u8c<23>(r);
    t.daddr = rec_raw32c<30>(r);
    t.saddr = rec_raw32c<26>(r);
    t.dport = t.sport = 0;
    const int off = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
    int64_t slot;
    int ret = ct_lookup4(ep.ct4, t, r, off, CT_INGRESS, now, p.flags, slot, a);
    if (ret < 0) return ret;
    ct_out = (uint8_t)ret;
    int verdict = policy_ingress(ep.policy, p.flags, r.len, src_label, t.dport, t.nexthdr, a);
    if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
        if (ret == CT_ESTABLISHED) { dev_kill<Ct4Spec>(ep.ct4, slot); a.nu++; }   // ct_delete4
        return DROP_POLICY;
    }
    if (skip_proxy) verdict = 0;
    if (ret == CT_NEW) {
        const int c = ct_create4_ingress(ep.ct4, t, r.len, src_label, now);
        a.nu += 2;
        if (c < 0 || c == TC_ACT_SHOT) return c;
    }
    if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
        proxy = (uint16_t)verdict;                                 // ipv4_redirect_to_host_port
        return TC_ACT_REDIRECT;                                    // redirect(HOST_IFINDEX)
    }
    return ifindex_nz ? TC_ACT_REDIRECT : TC_ACT_OK;
}

__device__ __forceinline__ bool is_err(int x) { return x < 0 || x == TC_ACT_SHOT; }   // common.h:231

// stage 1: XDP prefilter + from_netdev/handle_ipv4 up to the tail call into the
// endpoint's policy program; packets reaching it join their address-pair group.
__global__ void __launch_bounds__(BLOCK) k_netdev_front(DpParams p, BatchDev b, OutDev o, GroupScratch g,
                                                        int with_prefilter)
{
    __shared__ LdsMetrics lm;
    lm_init(lm);
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        Rec r;
        rec_load(r, b, i, 4);
        Acct a{0, 0};
        uint8_t xv = XDP_PASS;
        int32_t ret = TC_ACT_OK;
        uint32_t ident = 0;
        bool staged = false;
        if (with_prefilter) xv = xdp_verdict(p, r, a);
        if (xv == XDP_PASS) {
            bool skip_proxy = false;
            uint32_t identity = 0;
            if (p.flags & F_FROM_HOST) identity = identity_from_mark(b.mark ? b.mark[i] : 0u, skip_proxy);
            ident = identity;
            const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
            if (eth == 0x0008u) {
                int h;                                            // handle_ipv4 (bpf_netdev.c:357-453)
                if (r.len < 34) {
                    h = DROP_INVALID;
                } else {
                    const int l4 = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
                    const uint32_t nexthdr = rec_u8c<23>(r);
                    uint32_t secctx = WORLD_ID;
                    if (identity < HEALTH_ID) {
                        const uint32_t lab = ipcache4(p, rec_raw32c<26>(r), a);
                        if (lab && lab != CLUSTER_ID && lab != HOST_ID) identity = lab;
                    }
                    ident = identity;
                    h = TC_ACT_OK;
                    if (p.flags & F_FROM_HOST) {
                        secctx = identity;
                        if (nexthdr == 6 || nexthdr == 17) {      // reverse_proxy port load
                            const int c = rec_chk(r, l4, 4);
                            if (c) h = c == E_TRUNC ? E_TRUNC : DROP_CT_INVALID_HDR;
                        }
                    }
                    uint32_t iv;
                    if (h == TC_ACT_OK && lxc4_find(p, rec_raw32c<30>(r), iv, a)) {
                        if (iv & (1u << 16)) {
                            h = TC_ACT_OK;                        // ENDPOINT_F_HOST
                        } else if (rec_u8c<22>(r) <= 1) {
                            h = DROP_INVALID;                     // ipv4_dec_ttl
                        } else {
                            const uint32_t e = p.ep_of_lxc ? p.ep_of_lxc[iv & 0xFFFFu] : 0u;
                            if (!e) {
                                h = DROP_MISSED_TAIL_CALL;
                            } else {
                                staged = true;                    // -> tail_ipv4_policy
                                g.secctx[i] = secctx;
                                g.meta[i] = (e - 1) | (skip_proxy ? 1u << 16 : 0u) | ((iv >> 17) & 1u) << 17;
                                const EpDev &ep = p.eps[e - 1];
                                const uint32_t sa = rec_raw32c<26>(r), da = rec_raw32c<30>(r);
                                const uint32_t lo = sa < da ? sa : da, hi = sa < da ? da : sa;
                                uint64_t gh = mix64(((uint64_t)lo << 32 | hi) ^ ((uint64_t)ep.ct_id << 17));
                                const uint32_t h32 = (uint32_t)gh | 1u;
                                const unsigned long long tagged = (unsigned long long)g.epoch << 32 | h32;
                                uint32_t s = (uint32_t)(gh >> 32) & g.cap_mask;
                                for (;;) {
                                    unsigned long long cur = __hip_atomic_load(&g.table[2 * s], __ATOMIC_RELAXED,
                                                                               __HIP_MEMORY_SCOPE_AGENT);
                                    if (cur == tagged) break;
                                    if ((uint32_t)(cur >> 32) != g.epoch) {
                                        if (__hip_atomic_compare_exchange_strong(&g.table[2 * s], &cur, tagged,
                                                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                                 __HIP_MEMORY_SCOPE_AGENT))
                                            break;
                                        if (cur == tagged) break;
                                        if ((uint32_t)(cur >> 32) != g.epoch) continue;
                                    }
                                    s = (s + 1) & g.cap_mask;
                                }
                                const unsigned long long prev = __hip_atomic_exchange(
                                    &g.table[2 * s + 1], (unsigned long long)g.epoch << 32 | i, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
                                g.gslot[i] = s;
                                g.next[i] = (uint32_t)(prev >> 32) == g.epoch ? (uint32_t)prev : NONE;
                            }
                        }
                    }
                }
                if (!staged) {
                    if (h == E_TRUNC) ret = h;
                    else if (is_err(h)) { lm_add(lm, h, r.len); ret = TC_ACT_SHOT; }   // tail_handle_ipv4
                    else ret = h;
                }
            }
        }
        if (!staged) {
            g.gslot[i] = NONE;
            if (o.ret) o.ret[i] = ret;
            if (o.ct) o.ct[i] = CT_NONE;
            if (o.proxy) o.proxy[i] = 0;
            store_out(o, i, a);
        } else {
            if (o.nl) o.nl[i] = (uint8_t)a.nl;                  // stage 2 adds its own
            if (o.nu) o.nu[i] = (uint8_t)a.nu;
        }
        if (o.xdp) o.xdp[i] = xv;
        if (o.identity) o.identity[i] = ident;
    }
    lm_flush(lm, p.metrics, METRIC_INGRESS);
}

__device__ __forceinline__ void stage2_one(const DpParams &p, const BatchDev &b, const OutDev &o,
                                           const GroupScratch &g, uint32_t i, uint32_t now, LdsMetrics &lm)
{
    Rec r;
    rec_load(r, b, i, 3);
    const uint32_t meta = g.meta[i];
    const EpDev &ep = p.eps[meta & 0xFFFFu];
    Acct a{o.nl ? o.nl[i] : 0u, o.nu ? o.nu[i] : 0u};
    uint8_t ct = CT_NONE;
    uint16_t proxy = 0;
    int ret = ipv4_policy(p, ep, r, g.secctx[i], (meta >> 16) & 1u, (meta >> 17) & 1u, now, ct, proxy, a);
    if (ret != E_TRUNC && is_err(ret)) {                         // tail_ipv4_policy: send_drop_notify
        lm_add(lm, ret, r.len);
        ret = TC_ACT_SHOT;
    }
    if (o.ret) o.ret[i] = ret;
    if (o.ct) o.ct[i] = ct;
    if (o.proxy) o.proxy[i] = proxy;
    store_out(o, i, a);
}

constexpr int GMAX = 16;

// stage 2: conntrack + policy, each address-pair group by one lane in packet order
__global__ void __launch_bounds__(BLOCK) k_ct_stage(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsMetrics lm;
    lm_init(lm);
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        const uint32_t s = g.gslot[i];
        if (s == NONE || g.next[i] != NONE) continue;              // not staged / not the group's first inserter
        const uint32_t head = (uint32_t)g.table[2 * s + 1];
        if (head == i) { stage2_one(p, b, o, g, i, now, lm); continue; }
        // collect the group's members and run them in ascending packet order
        uint32_t m[GMAX];
        int cnt = 0;
        bool overflow = false;
        for (uint32_t x = head; x != NONE; x = g.next[x]) {
            if (cnt == GMAX) { overflow = true; break; }
            int pos = 0;
#pragma unroll
            for (int j = 0; j < GMAX; ++j) pos += (j < cnt && m[j] < x) ? 1 : 0;
#pragma unroll
            for (int j = GMAX - 1; j >= 0; --j) {
                const uint32_t left = j > 0 ? m[j - 1] : 0u;
                m[j] = (j < pos) ? m[j] : (j == pos ? x : left);
            }
            ++cnt;
        }
        if (!overflow) {
#pragma unroll 1
            for (int j = 0; j < GMAX; ++j) {
                if (j >= cnt) break;
                uint32_t v = m[0];
#pragma unroll
                for (int q = 1; q < GMAX; ++q) v = (q == j) ? m[q] : v;
                stage2_one(p, b, o, g, v, now, lm);
            }
        } else {
            uint32_t last = 0;
            bool first = true;
            for (;;) {                                             // repeated minimum scan
                uint32_t best = NONE;
                for (uint32_t x = head; x != NONE; x = g.next[x])
                    if ((first || x > last) && x < best) best = x;
                if (best == NONE) break;
                stage2_one(p, b, o, g, best, now, lm);
                last = best;
                first = false;
            }
        }
    }
    lm_flush(lm, p.metrics, METRIC_INGRESS);
}

// ------------------------------------------------------------------ CT map API
// Single-element BPF_MAP_{LOOKUP,UPDATE,DELETE}_ELEM on a device-resident CT table
// (the agent side of pkg/maps/ctmap: GC deletes, dumps, restores).
__global__ void k_ct_op(HashTable t, int op, uint64_t flags, uint32_t *io)
{
    if (threadIdx.x || blockIdx.x) return;
    uint32_t key[4] = {io[0], io[1], io[2], io[3]};
    int rc = 0;
    int64_t s = dev_find<Ct4Spec>(t, key, nullptr);
    if (op == 0) {
        if (s < 0) rc = -ENOENT;
        else {
            CtE e;
            ct_load(t, s, e);
            for (int k = 0; k < 16; ++k) io[4 + k] = e.w[k];
        }
    } else if (op == 1) {
        if (s >= 0 && flags == 1) rc = -EEXIST;
        else if (s < 0 && flags == 2) rc = -ENOENT;
        else {
            bool created;
            s = dev_upsert<Ct4Spec>(t, key, &created);
            if (s < 0) rc = -E2BIG;
            else {
                CtE e;
                for (int k = 0; k < 16; ++k) e.w[k] = io[4 + k];
                ct_store(t, s, e);
            }
        }
    } else {
        if (s < 0) rc = -ENOENT;
        else dev_kill<Ct4Spec>(t, s);
    }
    io[20] = (uint32_t)rc;
}

// compact every live entry (tag >= 3) into key/value arrays
__global__ void k_ct_scan(HashTable t, uint64_t nslots, uint32_t *keys, uint32_t *vals, uint32_t *count, uint32_t max)
{
    for (uint64_t x = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; x < nslots; x += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t b = x / Ct4Spec::SPB;
        const int sl = (int)(x % Ct4Spec::SPB);
        const uint32_t *bw = t.buckets + b * Ct4Spec::BW;
        const uint32_t tag = (bw[sl >> 2] >> (8 * (sl & 3))) & 0xFFu;
        if (tag < 3) continue;
        const uint32_t at = atomicAdd(count, 1u);
        if (at >= max) continue;
        for (int j = 0; j < 4; ++j) keys[at * 4 + j] = bw[Ct4Spec::KEY0 + sl * 4 + j];
        const uint32_t *v = reinterpret_cast<const uint32_t *>(t.vals + x * t.vstride);
        for (int j = 0; j < 16; ++j) vals[at * 16 + j] = v[j];
    }
}

// ------------------------------------------------------------------ host launchers
static inline int grid_for(uint32_t n)
{
    uint32_t g = (n + BLOCK - 1) / BLOCK;
    if (g > 2048) g = 2048;
    return g ? (int)g : 1;
}

int launch_xdp_prefilter(const DpParams &p, const BatchDev &b, const OutDev &o, hipStream_t s)
{
    if (!b.n) return 0;
    hipLaunchKernelGGL(k_xdp_prefilter, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// fold the per-chunk delta words into policy_entry.packets / .bytes
__global__ void __launch_bounds__(BLOCK) k_policy_fold(HashTable t, uint64_t nslots)
{
    for (uint64_t x = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; x < nslots; x += (uint64_t)gridDim.x * BLOCK) {
        const unsigned long long d = t.aux[x];
        if (!d) continue;
        unsigned long long *v = reinterpret_cast<unsigned long long *>(t.vals + x * t.vstride);
        v[1] += d >> 39;
        v[2] += d & ((1ull << 39) - 1);
        t.aux[x] = 0;
    }
}

int launch_policy_fold(const HashTable &pol, hipStream_t s)
{
    if (!pol.buckets || !pol.vals || !pol.aux) return 0;
    const uint64_t slots = (pol.mask + 1) * pol.spb;
    uint64_t g = (slots + BLOCK - 1) / BLOCK;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_policy_fold, dim3((uint32_t)g), dim3(BLOCK), 0, s, pol, slots);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_policy_ingress(const DpParams &p, int ep, const BatchDev &b, const OutDev &o, hipStream_t s)
{
    if (!b.n) return 0;
    const uint32_t grid = (b.n + PPT * BLOCK - 1) / (PPT * BLOCK);
    hipLaunchKernelGGL(k_policy_ingress, dim3(grid), dim3(BLOCK), 0, s, p, ep, b, o);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_netdev_ingress(const DpParams &p, const BatchDev &b, uint32_t now, int with_prefilter, const OutDev &o,
                          const GroupScratch &g, hipStream_t s)
{
    if (!b.n) return 0;
    hipLaunchKernelGGL(k_netdev_front, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, with_prefilter);
    if (hipGetLastError() != hipSuccess) return -5;
    hipLaunchKernelGGL(k_ct_stage, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, now);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ct_op(const HashTable &t, int op, uint64_t flags, uint32_t *io_dev, hipStream_t s)
{
    hipLaunchKernelGGL(k_ct_op, dim3(1), dim3(64), 0, s, t, op, flags, io_dev);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ct_scan(const HashTable &t, uint64_t nb, uint32_t *out_keys, uint32_t *out_vals, uint32_t *count,
                   uint32_t max, hipStream_t s)
{
    const uint64_t slots = nb * Ct4Spec::SPB;
    uint64_t g = (slots + BLOCK - 1) / BLOCK;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_ct_scan, dim3((uint32_t)g), dim3(BLOCK), 0, s, t, slots, out_keys, out_vals, count, max);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cv
