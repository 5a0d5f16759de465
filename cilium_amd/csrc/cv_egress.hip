// cv_egress.hip — gfx950 kernels of the from-container (egress) path, config 5.
//
// Restates bpf_lxc.c handle_ingress (:672-716) -> tail_handle_ipv4 /
// tail_handle_ipv6 -> handle_ipv4_from_lxc (:402-649) / ipv6_l3_from_lxc
// (:82-352) with lb4/lb6 service lookup and lb{4,6}_local (lib/lb.h), egress
// conntrack and policy, and local delivery into the destination endpoint's
// handle_policy (:1003-1038) -> ipv{4,6}_policy, direct routing (no ENCAP_IFINDEX),
// over a batch of frame records in HBM.  One lane = one packet.
//
// Batch semantics are those of one CPU running the packets in order.  Conntrack
// work is split in two disjoint key sets that commute:
//   * service entries (tuple flags with TUPLE_F_SERVICE), touched only by
//     lb{4,6}_local: k_lb_stage runs them grouped by (source, VIP) pair;
//   * all other entries: k_egress_ct runs them grouped by connected components of
//     the address pairs a packet can touch — its egress tuple, the NATed tuple a
//     service create writes, the pair its local delivery sees after rewrites and the
//     pairs a reverse-NAT of an entry it reads or creates can lead to — built by
//     k_egress_pairs (lock-free union-find), keyed by component in k_group_link and
//     grouped by binning (launch_gbin_groups).
// Within a group packets run in packet order; groups share no entry.
#include "cv_dev.hpp"

namespace cv {

// conntrack reads of the egress stages: plain loads, with the CU's L1 dropped after
// the lane's own in-place bucket changes (creates, deletes) so that its later lookups
// see them (see ld_tags); agent-scope loads on every read measured 3-5 % slower
constexpr bool EGF = false;
__device__ __forceinline__ void eg_changed() { l1_inv(); }


int grid_for(uint32_t n);

// occupancy knobs of the egress stages (measurements: 0 leaves the choice to the compiler)
#ifndef CV_LB_WAVES
#define CV_LB_WAVES 0
#endif
#ifndef CV_PAIRS_WAVES
#define CV_PAIRS_WAVES 0
#endif
#ifndef CV_EFRONT_WAVES
#define CV_EFRONT_WAVES 0
#endif
#define CV_WAVES_ATTR(w) __attribute__((amdgpu_waves_per_eu((w) ? (w) : 1, (w) ? 8 : 10)))


// egress scratch words (GroupScratch::eg, EG_WORDS per packet)
enum : uint32_t {
    EG_STAGE = 0x3u, EG_V6 = 0x4u, EG_LOOPBACK = 0x8u, EG_SVC = 0x10u, EG_DPORT_RW = 0x20u,
    EG_NAT_DEFER = 0x40u,       // the NATed tuple's pair is read by no packet of the launch
};
enum : uint32_t { STAGE_DONE = 0, STAGE_LB = 1, STAGE_CT = 2 };

// A dense word per packet (GroupScratch::ifx, which otherwise only the netdev path
// uses) with what the grouping passes after k_egress_pairs test on every packet,
// so they stream 4 B per packet instead of its 64-B scratch line: the conntrack queue
// (IPv6), a NAT-tuple writer to place (k_egress_nat), a deferred NAT write made
// (k_nat_group).  Written by k_egress_pairs for every packet, BIT_NAT_DONE by the
// packet's own lane in k_egress_ct.
enum : uint32_t { BIT_V6 = 1, BIT_NAT_CAND = 2, BIT_NAT_DONE = 4, BIT_NAT_DEFER = 8 };
constexpr uint64_t SALT_SVC4 = 0x5356433400000000ULL, SALT_SVC6 = 0x5356433600000000ULL,
                   SALT_CT4 = 0x4354340000000000ULL, SALT_CT6 = 0x4354360000000000ULL,
                   SALT_NAT = 0x4E41540000000000ULL, SALT_SELF = 0x53454C4600000000ULL;

// The NATed tuple a non-loopback service create writes is a self-pair key (backend,
// backend, the flow's ports).  A packet can read it only through a lookup key of the
// same pair, protocol and (unordered) ports, so readers of self-pair keys register a
// node keyed by (address, port pair, protocol) and a NAT writer joins a group only
// through that node (k_egress_nat).  proto = 0x100: "any ports" (a rewritten key).
__device__ __forceinline__ uint32_t port_sig(const Tuple4 &t)
{
    const uint32_t a = t.sport & 0xFFFFu, c = t.dport & 0xFFFFu;
    return a < c ? (a | c << 16) : (c | a << 16);
}

__device__ __forceinline__ uint64_t self_hash(uint32_t x, uint32_t sig, uint32_t proto)
{
    return mix64(((uint64_t)x << 32 | sig) ^ ((uint64_t)proto << 52) ^ SALT_SELF);
}

struct EgOut {                  // per-packet results on the way to the outputs
    int32_t ret, reason;
    uint32_t dst;
    uint8_t ct;
    uint16_t proxy;
};

// Egress admission (cv_ctx.cpp lxc_admitted): a packet's creates of new conntrack
// entries draw on ONE budget across its service, conntrack and delivery stages, in that
// order (the order of its map_update_elem calls in the reference).  A stage takes the
// budget left from p.eg_left, hands back what it did not use, and adds to the packet's
// intent byte the creates it tried (a failing one included: the reference's failing
// map_update_elem ends the packet) and the deletes it made.  `flush` hands over before
// an inline delivery of the same packet.  With many CT maps (p.eg_left2) the local
// delivery (slot 1) draws on a budget of its own -- its creates and delete go to the
// destination's map -- and records the destination endpoint (dep); every stage saves a
// CT slot before its first write in the pass (p.snap).
struct EgAdm {
    const DpParams &p;
    uint32_t i;
    Acct &a;
    bool on, two;
    // sn: the kernel instance saves CT slots (MetT::SN; the others compile it out)
    __device__ EgAdm(const DpParams &pp, uint32_t ii, Acct &aa, bool live, bool sn, int slot = 0, uint32_t dep = 0)
        : p(pp), i(ii), a(aa), on(live && pp.eg_left), two(sn && slot && pp.eg_left2)   // (many maps: SN only)
    {
        if (on) {
            a.budget = (two ? p.eg_left2 : p.eg_left)[i];
            a.tried = a.killed = 0;
            if (sn) {
                a.snap = p.snap;
                a.spkt = i;
                a.scnt = p.snap->cnt[i];
            }
            if (two) p.eg_dst[i] = (uint16_t)dep;
        }
    }
    __device__ void flush()
    {
        if (!on) return;
        if (a.snap) a.snap->cnt[i] = (uint8_t)a.scnt;
        uint8_t *intent = two ? p.eg_intent2 : p.eg_intent;
        (two ? p.eg_left2 : p.eg_left)[i] = (uint8_t)a.budget;
        intent[i] = (uint8_t)(intent[i] + a.tried + (a.killed << 3));
        on = false;
    }
    __device__ ~EgAdm() { flush(); }
};

__device__ __forceinline__ void eg_final(const OutDev &o, uint32_t i, const EgOut &r, const Acct &a)
{
    if (o.ret) o.ret[i] = r.ret;
    if (o.reason) o.reason[i] = r.reason;
    if (o.identity) o.identity[i] = r.dst;
    if (o.ct) o.ct[i] = r.ct;
    if (o.proxy) o.proxy[i] = r.proxy;
    if (o.xdp) o.xdp[i] = 0;
    store_out(o, i, a);
}

// The final outputs of a packet a scattered stage (service, conntrack, delivery: lanes
// take packets in group order) finishes, as ONE 16-B store into its g.res slot instead
// of a store per output array -- each a random line of HBM -- written out in packet
// order by k_out_unpack: {identity, ret | -reason << 8 | ct << 16 | RES_DONE,
// proxy | nl << 16 | nu << 24, 0} (ret is one of the small TC_ACT_* / E_* codes, reason
// a DROP_* code or 0)
constexpr uint32_t RES_DONE = 1u << 24;
__device__ __forceinline__ void eg_done(const GroupScratch &g, uint32_t i, const EgOut &r, const Acct &a)
{
    g.res[i] = make_uint4(r.dst, ((uint32_t)r.ret & 0xFFu) | ((uint32_t)(-r.reason) & 0xFFu) << 8 |
                                     (uint32_t)r.ct << 16 | RES_DONE,
                          (uint32_t)r.proxy | (a.nl & 0xFFu) << 16 | (a.nu & 0xFFu) << 24, 0u);
}

__global__ void __launch_bounds__(BLOCK) k_out_unpack(OutDev o, GroupScratch g, uint32_t n)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const uint4 r = g.res[i];
        if (!(r.y & RES_DONE)) continue;                          // (finished in the front)
        if (o.ret) o.ret[i] = (int32_t)(int8_t)(r.y & 0xFFu);
        if (o.reason) o.reason[i] = -(int32_t)((r.y >> 8) & 0xFFu);
        if (o.identity) o.identity[i] = r.x;
        if (o.ct) o.ct[i] = (uint8_t)(r.y >> 16);
        if (o.proxy) o.proxy[i] = (uint16_t)r.z;
        if (o.xdp) o.xdp[i] = 0;
        if (o.nl) o.nl[i] = (uint8_t)(r.z >> 16);
        if (o.nu) o.nu[i] = (uint8_t)(r.z >> 24);
    }
}

template <bool FULL>
__device__ __forceinline__ EpDev eg_src4(const DpParams &p, uint32_t idx)
{
    if constexpr (FULL) return G(p.eps)[idx];
    return ep_netdev4<false>(p, idx);                             // (the plain LB stage reads the CT map only)
}

// The service stage's input state of a packet (the front parsed it anyway), in the
// packet's 64-B line of g.est (k_egress_pairs later overwrites it with the conntrack
// stage's): IPv4 d0 skb4_pack(s), d1 {w4, chk, 0, 0}; IPv6 d0 saddr, d1 daddr, d2 {len,
// nexthdr | type << 8 | tflags << 16 | l4off << 24, ports, chk}; both d3 {eg[1], eg[2]}
__device__ __forceinline__ void lb_pack4(const Skb4 &s, uint32_t e1, uint32_t e2, uint4 *d)
{
    uint32_t w4, chk;
    d[0] = skb4_pack(s, w4, chk);
    d[1] = make_uint4(w4, chk, 0u, 0u);
    d[3] = make_uint4(e1, e2, 0u, 0u);
}

__device__ __forceinline__ void lb_pack6(const Skb6 &s, uint32_t e1, uint32_t e2, uint4 *d)
{
    d[0] = make_uint4(s.saddr[0], s.saddr[1], s.saddr[2], s.saddr[3]);
    d[1] = make_uint4(s.daddr[0], s.daddr[1], s.daddr[2], s.daddr[3]);
    d[2] = make_uint4(s.len, (s.nexthdr & 0xFFu) | (s.h.type & 0xFFu) << 8 | (s.h.tflags & 0xFFu) << 16 |
                                 ((uint32_t)s.l4off & 0xFFu) << 24,
                      (s.h.p0 & 0xFFFFu) | s.h.p2 << 16,
                      chk2(s.h.c1) | chk2(s.h.c14) << 2 | chk2(s.h.c4) << 4 | chk2(s.h.c2a) << 6 | chk2(s.h.c2b) << 8);
    d[3] = make_uint4(e1, e2, 0u, 0u);
}

__device__ __forceinline__ void skb6_unpack(const uint4 &d0, const uint4 &d1, const uint4 &d2, uint32_t stride, Skb6 &s)
{
    s.saddr[0] = d0.x; s.saddr[1] = d0.y; s.saddr[2] = d0.z; s.saddr[3] = d0.w;
    s.daddr[0] = d1.x; s.daddr[1] = d1.y; s.daddr[2] = d1.z; s.daddr[3] = d1.w;
    s.len = d2.x;
    s.nexthdr = d2.y & 0xFFu;
    s.l4off = (int)(d2.y >> 24);
    s.avail = stride;
    s.h.type = (d2.y >> 8) & 0xFFu;
    s.h.tflags = (d2.y >> 16) & 0xFFu;
    s.h.p0 = d2.z & 0xFFFFu;
    s.h.p2 = d2.z >> 16;
    s.h.c1 = unchk2(d2.w & 3u);
    s.h.c14 = unchk2((d2.w >> 2) & 3u);
    s.h.c4 = unchk2((d2.w >> 4) & 3u);
    s.h.c2a = unchk2((d2.w >> 6) & 3u);
    s.h.c2b = unchk2((d2.w >> 8) & 3u);
    s.hoplimit = (d2.w >> 16) & 0xFFu;
}

// a lane's 64 B at dst + 64 * lane (the wave's 64 consecutive lines) through LDS as four
// coalesced 1-KiB stores; all 64 lanes, wave-uniform (`st`: 256 uint4)
__device__ __forceinline__ void wave_store64(uint4 *dst, const uint4 *v, uint4 *st)
{
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) st[k * 64 + lane] = v[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int chunk = c * 64 + lane;                          // line chunk / 4, part chunk % 4
        dst[chunk] = st[(chunk & 3) * 64 + (chunk >> 2)];
    }
    __builtin_amdgcn_wave_barrier();
}

// a local delivery handed over to k_egress_deliver (see there)
__device__ __forceinline__ void del_list(const GroupScratch &g, bool v6, uint32_t i)
{
    const uint32_t at = wave_append(&g.cursor[del_ctr(v6, g.pos)], true);
    g.single[at] = i;
}

// tail_handle_ipv{4,6} / handle_ingress: IS_ERR -> send_drop_notify(METRIC_EGRESS)
template <class M>
__device__ __forceinline__ void eg_drop(const DpParams &p, EgOut &r, int32_t code, uint32_t len, M &m)
{
    if (code == E_TRUNC || code == E_PUNT) { r.ret = code; return; }
    m.drop(code, len, METRIC_EGRESS);
    notify_drop(p, m, code, len, m.src_id, m.src_label, 0, 0, 0);   // send_drop_notify(SECLABEL, 0, 0, 0)
    r.reason = code;
    r.ret = TC_ACT_SHOT;
}

__device__ __forceinline__ bool mac_eq(uint32_t w0, uint32_t h1, const uint32_t *mac)
{
    return w0 == mac[0] && h1 == (mac[1] & 0xFFFFu);
}

// ================================================================== front
// handle_ingress dispatch + the from-container prologue up to lb{4,6}_lookup_service.
// Returns STAGE_LB (service found), STAGE_CT, or STAGE_DONE with r filled.
template <int NW, class M>
__device__ __forceinline__ uint32_t front_one(const DpParams &p, const EpDev &ep, const RecT<NW> &r, uint32_t *eg,
                                              EgOut &res, Acct &a, M &m)
{
    const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
    int ret;
    if (p.flags & F_DROP_ALL) {
        if (eth == 0x0608u) { res.ret = E_PUNT; return STAGE_DONE; }   // ARP responder tail call
        eg_drop(p, res, DROP_POLICY, r.len, m);
        return STAGE_DONE;
    }
    if (eth == 0x0008u) {
        if (!ep.ipv4) { eg_drop(p, res, DROP_MISSED_TAIL_CALL, r.len, m); return STAGE_DONE; }
        // handle_ipv4_from_lxc (bpf_lxc.c:402-446)
        if (r.len < 34) { eg_drop(p, res, DROP_INVALID, r.len, m); return STAGE_DONE; }
        if (!mac_eq(rec_raw32c<6>(r), rec_raw16c<10>(r), ep.mac)) ret = DROP_INVALID_SMAC;
        else if (!mac_eq(rec_raw32c<0>(r), rec_raw16c<4>(r), ep.node_mac)) ret = DROP_INVALID_DMAC;
        else if (rec_raw32c<26>(r) != ep.ipv4) ret = DROP_INVALID_SIP;
        else ret = 0;
        if (ret) { eg_drop(p, res, ret, r.len, m); return STAGE_DONE; }
        const uint32_t nexthdr = rec_u8c<23>(r);
        const int off = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
        const L4Hdr h = l4_read<34>(r, off);
        uint32_t dport = 0;
        if (nexthdr == 6 || nexthdr == 17) {                      // lb4_extract_key / extract_l4_port
            if (h.c2b) { eg_drop(p, res, chk_err(h.c2b, E_FAULT), r.len, m); return STAGE_DONE; }
            dport = h.p2;
        } else if (nexthdr != 1) {
            return STAGE_CT;                                      // DROP_UNKNOWN_L4: skip_service_lookup
        }
        if (!p.lb4.buckets) return STAGE_CT;
        // lb4_lookup_service (lb.h:604-635), LB_L4 + LB_L3
        const uint32_t daddr = rec_raw32c<30>(r);
        uint32_t k[2], v[3];
        if (dport) {
            k[0] = daddr; k[1] = dport;
            a.nl++;
            if (dev_find<Lb4Spec>(p.lb4, k, v) >= 0 && (v[1] >> 16)) {
                eg[1] |= dport << 16; eg[2] = v[1] >> 16;
                return STAGE_LB;
            }
            dport = 0;
        }
        k[0] = daddr; k[1] = 0;
        a.nl++;
        if (dev_find<Lb4Spec>(p.lb4, k, v) >= 0 && (v[1] >> 16)) {
            eg[2] = v[1] >> 16;
            return STAGE_LB;
        }
        return STAGE_CT;
    }
    if (eth == 0xDD86u) {
        if constexpr (NW < 32) {
            res.ret = E_TRUNC;                                    // IPv6 needs 128-B records
            return STAGE_DONE;
        } else {
            if (!ep.ct6.buckets) { eg_drop(p, res, DROP_MISSED_TAIL_CALL, r.len, m); return STAGE_DONE; }
            // handle_ipv6 (bpf_lxc.c:360-387) + ipv6_l3_from_lxc (:82-125)
            if (r.len < 54) { eg_drop(p, res, DROP_INVALID, r.len, m); return STAGE_DONE; }
            eg[0] |= EG_V6;
            if (rec_u8c<20>(r) == 58) {                          // icmp6_handle (icmp6.h:390-412)
                if (r.len < 62) { eg_drop(p, res, DROP_INVALID, r.len, m); return STAGE_DONE; }
                const uint32_t type = rec_u8c<54>(r);
                const uint32_t da[4] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r)};
                if (type == 135 || (type == 128 && eq4(da, p.router6))) { res.ret = E_PUNT; return STAGE_DONE; }
            }
            const uint32_t sa[4] = {rec_raw32c<22>(r), rec_raw32c<26>(r), rec_raw32c<30>(r), rec_raw32c<34>(r)};
            if (!mac_eq(rec_raw32c<6>(r), rec_raw16c<10>(r), ep.mac)) ret = DROP_INVALID_SMAC;
            else if (!mac_eq(rec_raw32c<0>(r), rec_raw16c<4>(r), ep.node_mac)) ret = DROP_INVALID_DMAC;
            else if (!eq4(sa, ep.ipv6)) ret = DROP_INVALID_SIP;
            else ret = 0;
            if (ret) { eg_drop(p, res, ret, r.len, m); return STAGE_DONE; }
            uint32_t nexthdr;
            const int hl = ipv6_hdrlen(r, nexthdr);
            if (hl < 0) { eg_drop(p, res, hl, r.len, m); return STAGE_DONE; }
            const int off = 14 + hl;
            const L4Hdr h = l4_read<54>(r, off);
            uint32_t dport = 0;
            if (nexthdr == 6 || nexthdr == 17) {
                if (h.c2b) { eg_drop(p, res, chk_err(h.c2b, E_FAULT), r.len, m); return STAGE_DONE; }
                dport = h.p2;
            } else if (nexthdr != 58 && nexthdr != 1) {
                return STAGE_CT;
            }
            if (!p.lb6.buckets) return STAGE_CT;
            uint32_t k[5] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r), 0};
            uint32_t v[6];
            if (dport) {                                          // lb6_lookup_service (lb.h:351-380)
                k[4] = dport;
                a.nl++;
                if (dev_find<Lb6Spec>(p.lb6, k, v) >= 0 && (v[4] >> 16)) {
                    eg[1] |= dport << 16; eg[2] = v[4] >> 16;
                    return STAGE_LB;
                }
            }
            k[4] = 0;
            a.nl++;
            if (dev_find<Lb6Spec>(p.lb6, k, v) >= 0 && (v[4] >> 16)) {
                eg[2] = v[4] >> 16;
                return STAGE_LB;
            }
            return STAGE_CT;
        }
    }
    if (eth == 0x0608u) { res.ret = E_PUNT; return STAGE_DONE; }
    eg_drop(p, res, DROP_UNKNOWN_L3, r.len, m);
    return STAGE_DONE;
}

template <int NW, bool EV>
__global__ void __launch_bounds__(BLOCK) CV_WAVES_ATTR(CV_EFRONT_WAVES) k_egress_front(DpParams p, BatchDev b, const uint16_t *src_ep, uint32_t ep0,
                                                        OutDev o, GroupScratch g)
{
    __shared__ LdsMetrics lm;
    __shared__ uint4 stage[BLOCK / 64][16 * NW];                  // cooperative record loads
    uint4 *st = stage[threadIdx.x >> 6];
    using M = MetT<EV>;
    M m;
    met_init(m, lm);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < b.n; i0 += gridDim.x * BLOCK) {
        const uint32_t i = i0 + lane;
        RecT<NW> r;
        const bool full = i0 + 64 <= b.n && b.stride == 4 * NW;  // (wave-uniform)
        if (full) rec_load_coop(r, b, i0, st);
        else if (i < b.n) rec_load(r, b, i, NW / 4);
        if (i >= b.n) continue;
        uint4 es[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) es[k] = make_uint4(0u, 0u, 0u, 0u);
        Acct a{0, 0};
        a.ctu = ct_unit(p);
        EgOut res{TC_ACT_OK, 0, 0, CT_NONE, 0};
        uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
        const uint32_t e = src_ep ? src_ep[i] : ep0;
        if (M::EV && o.frames) frame_copy(b.frames + (size_t)i * b.stride, o.frames + (size_t)i * b.stride, b.stride);
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        m.src_id = e < p.n_eps ? G(p.eps)[e].lxc_id : 0u;
        m.src_label = e < p.n_eps ? G(p.eps)[e].seclabel : 0u;
        uint32_t egl[3] = {0u, e & 0xFFFFu, 0u};                 // eg[0..2], stored once below
        uint32_t stage;
        if (e >= p.n_eps) {
            res.ret = DROP_MISSED_TAIL_CALL;                      // no program for the source: nothing ran
            stage = STAGE_DONE;
        } else {
            const EpDev ep = G(p.eps)[e];                           // handle_ingress: send_trace_notify(FROM_LXC)
            notify_trace(p, m, TRACE_FROM_LXC, r.len, ep.lxc_id, ep.seclabel, 0, 0, 0, 0, true);
            stage = front_one(p, ep, r, egl, res, a, m);
        }
        egl[0] |= stage;
        reinterpret_cast<uint4 *>(eg)[0] = make_uint4(egl[0], egl[1], egl[2], 0u);
        g.gslot[i] = NONE;
        g.hword[i] = 0;
        unsigned long long gk = 0;                                // the service group key (binned grouping)
        if (stage == STAGE_DONE) {
            eg_final(o, i, res, a);
        } else {
            store_out(o, i, a);
            if (stage == STAGE_LB) {                              // the (source, VIP) service group
                const uint32_t ct_id = G(p.eps)[e].ct_id;
                uint64_t gh;
                if (egl[0] & EG_V6) {
                    if constexpr (NW >= 32) {
                        const uint32_t sa[4] = {rec_raw32c<22>(r), rec_raw32c<26>(r), rec_raw32c<30>(r), rec_raw32c<34>(r)};
                        const uint32_t da[4] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r)};
                        gh = pair_hash6(sa, da, SALT_SVC6 ^ ct_id);
                    } else {
                        gh = 0;
                    }
                } else {
                    gh = pair_hash4(rec_raw32c<26>(r), rec_raw32c<30>(r), SALT_SVC4 ^ ct_id);
                }
                gk = (gh & ~3ull) | 2ull | ((egl[0] & EG_V6) ? 1ull : 0ull);
                // the service stage's input: the parsed skb and the scratch words it reads
                if (egl[0] & EG_V6) {
                    if constexpr (NW >= 32) lb_pack6(skb6_from(r), egl[1], egl[2], es);
                } else {
                    lb_pack4(skb4_from(rec_head(r)), egl[1], egl[2], es);
                }
            }
        }
        g.pkey[i] = gk;
        g.res[i] = make_uint4(0u, 0u, 0u, 0u);                   // (RES_DONE clear: finished here or later)
        if (p.eg_left) {                                          // admission: this pass's budget, the intent's map
            p.eg_left[i] = stage == STAGE_DONE ? 0u : p.budget[i];
            p.eg_intent[i] = stage == STAGE_DONE ? 0u : ((egl[0] & EG_V6) ? 16u : 0u) | 32u;   // (32: runs on)
            if (p.eg_left2) {                                     // (the delivery's: budgets after the first pass's)
                p.eg_left2[i] = stage == STAGE_DONE ? 0u : p.budget[b.n + i];
                p.eg_intent2[i] = 0;
                p.eg_dst[i] = 0xFFFFu;
            }
        }
        if (!full && stage == STAGE_LB) {
#pragma unroll
            for (int k = 0; k < 4; ++k) g.est[(size_t)i * 4 + k] = es[k];
        }
        if (full) wave_store64(g.est + (size_t)i0 * 4, es, st);
    }
    met_flush(m, p.metrics);
}

// ================================================================== service stage
// lb4_local (lb.h:700-775) + lb4_xlate (:653-697) of one packet; the packet leaves
// with its translation in the scratch words, or final.
template <class M>
__device__ __forceinline__ void lb4_one(const DpParams &p, const BatchDev &b, const uint32_t *hash, uint32_t now,
                                        const OutDev &o, const GroupScratch &g, uint32_t i, M &m)
{
    const uint4 *d = g.est + (size_t)i * 4;
    const uint4 d0 = d[0], d1 = d[1], d3 = d[3];
    const Skb4 sk = skb4_unpack(d0, d1.x, d1.y & 0x3FFu, b.stride);
    uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
    const EpDev ep = eg_src4<M::EV>(p, d3.x & 0xFFFFu);
    m.pkt = b.base + i;
    m.hash = b.hash ? b.hash[i] : 0u;
    m.src_id = ep.lxc_id;
    m.src_label = ep.seclabel;
    Acct a{o.nl ? o.nl[i] : 0u, o.nu ? o.nu[i] : 0u, m.pc};
    a.ctu = ct_unit(p);
    EgAdm adm(p, i, a, true, M::SN);
    EgOut res{TC_ACT_OK, 0, 0, CT_NONE, 0};
    const uint32_t hsh = hash ? hash[i] : 0u;
    uint32_t key_dport = d3.x >> 16;
    const uint32_t count = d3.y & 0xFFFFu;
    const uint32_t saddr = sk.saddr, vip = sk.daddr;
    const int off = sk.l4off;
    L4Hdr h = sk.h;
    Tuple4 t;
    t.daddr = vip; t.saddr = saddr; t.nexthdr = sk.nexthdr; t.dport = t.sport = 0;
    CtState st{0, 0, 0, 0, 0, 0};
    int64_t slot;
    int ret = ct_lookup<false, EGF>(ep.ct4, t, h, CT_SERVICE, sk.len, now, p.flags, slot, &st, a);
    uint32_t k[2], v[3];
    bool have = false;
    if (ret == E_TRUNC) goto fin;
    if (ret == CT_NEW) {
        st.slave = hsh % count + 1;                               // lb4_select_slave
        const int c = ct_create<false>(ep.ct4, t, sk.len, CT_SERVICE, st, now, a, p.ct_guard, false, true);
        eg_changed();
        if (is_err(c)) { ret = DROP_NO_SERVICE; goto fin; }
    } else if (ret < 0) {
        ret = DROP_NO_SERVICE;
        goto fin;
    }
    k[0] = vip; k[1] = key_dport | st.slave << 16;                // lb4_lookup_slave
    a.nl++;
    have = dev_find<Lb4Spec>(p.lb4, k, v) >= 0;
    if (!have) {                                                  // backend gone: lb4_lookup_service with the slave key
        if (key_dport) {
            a.nl++;
            have = dev_find<Lb4Spec>(p.lb4, k, v) >= 0 && (v[1] >> 16);
            if (!have) { key_dport = 0; k[1] = st.slave << 16; }
        }
        if (!have) {
            a.nl++;
            have = dev_find<Lb4Spec>(p.lb4, k, v) >= 0 && (v[1] >> 16);
        }
        if (!have) { ret = DROP_NO_SERVICE; goto fin; }
        st.slave = hsh % (v[1] >> 16) + 1;
        uint32_t tk[4];                                           // ct_update4_slave
        t.key(tk);
        a.nl += a.ctu;
        const int64_t s2 = dev_find<Ct4Spec, EGF>(ep.ct4, tk, nullptr);
        if (s2 >= 0) {
            CtE e;
            snap_before<Ct4Spec>(a, ep.ct4, s2, SNAP_HOT);
            ct_load_hot<Ct4Spec>(ep.ct4, s2, e);                  // (w10: a hot word)
            const CtE e0 = e;
            e.w[10] = (e.w[10] & 0xFFFF0000u) | (st.slave & 0xFFFFu);
            ct_store_hot_diff<Ct4Spec>(ep.ct4, s2, e, e0);
            a.nu += a.ctu;
        }
    }
    {
        const uint32_t target = v[0], sport_svc = v[1] & 0xFFFFu;
        st.rev_nat = v[2] & 0xFFFFu;
        st.addr = target;
        uint32_t skb_saddr = saddr;
        if (saddr == target) {                                    // !DISABLE_LOOPBACK_LB
            skb_saddr = p.v4_loopback;
            st.loopback = 1;
            st.addr = p.v4_loopback;
            st.svc_addr = saddr;
        }
        const uint32_t tdaddr = st.loopback ? vip : target;
        uint32_t flags = STAGE_CT | EG_SVC | (st.loopback ? EG_LOOPBACK : 0u);
        const int coff = t.nexthdr == 6 ? 16 : t.nexthdr == 17 ? 6 : 0;   // lb4_xlate: the L4 checksum
        if (coff) {                                               // update by diff (pseudo header)
            const int c = len_chk(sk.len, b.stride, off + coff, 2);
            if (c) { ret = chk_err(c, DROP_CSUM_L4); goto fin; }
        }
        uint32_t ndport = 0;
        if (sport_svc && key_dport != sport_svc && (t.nexthdr == 6 || t.nexthdr == 17)) {
            if (h.c2b) { ret = chk_err(h.c2b, DROP_WRITE_ERROR); goto fin; }
            ndport = sport_svc;
            flags |= EG_DPORT_RW;
        }
        // eg[2]: the final lb4_key.dport | the rewritten port; eg[7]: the skb daddr after
        // lb4_xlate (three wide stores; eg[1] rewritten unchanged)
        uint4 *e4 = reinterpret_cast<uint4 *>(eg);
        e4[0] = make_uint4(flags, d3.x, ndport << 16 | (key_dport & 0xFFFFu), (st.rev_nat & 0xFFFFu) | st.slave << 16);
        e4[1] = make_uint4(st.addr, st.svc_addr, tdaddr, target);
        eg[8] = skb_saddr;
        store_out(o, i, a);
        return;
    }
fin:
    eg[0] = STAGE_DONE;
    eg_drop(p, res, ret, sk.len, m);
    eg_done(g, i, res, a);
}

// lb6_local (lb.h:426-483) + lb6_xlate (:386-424)
template <class M>
__device__ __forceinline__ void lb6_one(const DpParams &p, const BatchDev &b, const uint32_t *hash, uint32_t now,
                                        const OutDev &o, const GroupScratch &g, uint32_t i, M &m)
{
    const uint4 *d = g.est + (size_t)i * 4;
    const uint4 d3 = d[3];
    Skb6 s;
    skb6_unpack(d[0], d[1], d[2], b.stride, s);
    uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
    const EpDev ep = ep_uni6<M::EV>(p, d3.x & 0xFFFFu);          // (the plain instance reads the CT6 map only)
    m.pkt = b.base + i;
    m.hash = b.hash ? b.hash[i] : 0u;
    m.src_id = ep.lxc_id;
    m.src_label = ep.seclabel;
    Acct a{o.nl ? o.nl[i] : 0u, o.nu ? o.nu[i] : 0u, m.pc};
    a.ctu = ct_unit(p);
    EgAdm adm(p, i, a, true, M::SN);
    EgOut res{TC_ACT_OK, 0, 0, CT_NONE, 0};
    const uint32_t hsh = hash ? hash[i] : 0u;
    uint32_t key_dport = d3.x >> 16;
    const uint32_t count = d3.y & 0xFFFFu;
    Tuple6 t;
#pragma unroll
    for (int j = 0; j < 4; ++j) { t.daddr[j] = s.daddr[j]; t.saddr[j] = s.saddr[j]; }
    t.nexthdr = s.nexthdr; t.dport = t.sport = 0;
    CtState st{0, 0, 0, 0, 0, 0};
    int64_t slot;
    int ret = ct_lookup<true, EGF>(ep.ct6, t, s.h, CT_SERVICE, s.len, now, p.flags, slot, &st, a);
    uint32_t k[5] = {s.daddr[0], s.daddr[1], s.daddr[2], s.daddr[3], 0}, v[6];
    bool have = false;
    if (ret == E_TRUNC) goto fin;
    if (ret == CT_NEW) {
        st.slave = hsh % count + 1;
        const int c = ct_create<true>(ep.ct6, t, s.len, CT_SERVICE, st, now, a, p.ct_guard, false, true);
        eg_changed();
        if (is_err(c)) { ret = DROP_NO_SERVICE; goto fin; }
    } else if (ret < 0) {
        ret = DROP_NO_SERVICE;
        goto fin;
    }
    k[4] = key_dport | st.slave << 16;
    a.nl++;
    have = dev_find<Lb6Spec>(p.lb6, k, v) >= 0;
    if (!have) {
        if (key_dport) {
            a.nl++;
            have = dev_find<Lb6Spec>(p.lb6, k, v) >= 0 && (v[4] >> 16);
            if (!have) { key_dport = 0; k[4] = st.slave << 16; }
        }
        if (!have) {
            a.nl++;
            have = dev_find<Lb6Spec>(p.lb6, k, v) >= 0 && (v[4] >> 16);
        }
        if (!have) { ret = DROP_NO_SERVICE; goto fin; }
        st.slave = hsh % (v[4] >> 16) + 1;
        uint32_t tk[10];                                          // ct_update6_slave
        t.key(tk);
        a.nl += a.ctu;
        const int64_t s2 = dev_find<Ct6Spec, EGF>(ep.ct6, tk, nullptr);
        if (s2 >= 0) {
            CtE e;
            snap_before<Ct6Spec>(a, ep.ct6, s2, SNAP_HOT);
            ct_load_hot<Ct6Spec>(ep.ct6, s2, e);
            const CtE e0 = e;
            e.w[10] = (e.w[10] & 0xFFFF0000u) | (st.slave & 0xFFFFu);
            ct_store_hot_diff<Ct6Spec>(ep.ct6, s2, e, e0);
            a.nu += a.ctu;
        }
    }
    {
        const uint32_t sport_svc = v[4] & 0xFFFFu;
        st.rev_nat = v[5] & 0xFFFFu;
        uint32_t flags = STAGE_CT | EG_V6 | EG_SVC;
        {                                                         // lb6_xlate: the L4 checksum update by
            const int c = l4_csum_err6(s);                        // diff (any offset, ICMP's too)
            if (c) { ret = c; goto fin; }
        }
        uint32_t ndport = 0;
        if (sport_svc && key_dport != sport_svc && (t.nexthdr == 6 || t.nexthdr == 17)) {
            if (s.h.c2b) { ret = chk_err(s.h.c2b, DROP_WRITE_ERROR); goto fin; }
            ndport = sport_svc;
            flags |= EG_DPORT_RW;
        }
        uint4 *e4 = reinterpret_cast<uint4 *>(eg);                // (eg[2]: the final lb6_key.dport)
        e4[0] = make_uint4(flags, d3.x, ndport << 16 | (key_dport & 0xFFFFu), (st.rev_nat & 0xFFFFu) | st.slave << 16);
        eg[4] = 0; eg[5] = 0;
        e4[3] = make_uint4(v[0], v[1], v[2], v[3]);               // tuple daddr = skb daddr = target
        store_out(o, i, a);
        return;
    }
fin:
    eg[0] = STAGE_DONE;
    eg_drop(p, res, ret, s.len, m);
    eg_done(g, i, res, a);
}

// the service groups by member position, as the conntrack stage (position lists of the
// binned grouping; one launch per position)
template <bool V6, bool EV, bool SN = false>
__global__ void __launch_bounds__(BLOCK) CV_WAVES_ATTR(CV_LB_WAVES) k_lb_stage(DpParams p, BatchDev b, const uint32_t *hash, uint32_t now,
                                                    OutDev o, GroupScratch g, uint32_t pos)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;                                      // (here: the CT maps' live counts)
    using M = MetT<EV, SN>;
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    for_each_at(g, V6 ? Q_LB6 : Q_LB4, pos, [&](uint32_t x) {
        if constexpr (V6) lb6_one(p, b, hash, now, o, g, x, m);
        else lb4_one(p, b, hash, now, o, g, x, m);
    });
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// ================================================================== egress state of a packet
struct Eg4 {
    Skb4 s;
    Tuple4 t;                   // tuple before ct_lookup4(CT_EGRESS)
    CtState stn;                // ct_state_new from the service stage
};

__device__ __forceinline__ void eg4_state(const Rec &r, const uint32_t *eg, Eg4 &x)
{
    x.s = skb4_from(r);
    x.t.nexthdr = x.s.nexthdr;
    x.t.saddr = x.s.saddr;
    x.t.daddr = x.s.daddr;
    x.t.dport = x.t.sport = 0;
    x.stn = CtState{0, 0, 0, 0, 0, 0};
    if (eg[0] & EG_SVC) {
        x.t.daddr = eg[6];
        x.s.daddr = eg[7];
        x.s.saddr = eg[8];
        if (eg[0] & EG_DPORT_RW) x.s.h.p2 = eg[2] >> 16;
        x.stn.rev_nat = eg[3] & 0xFFFFu;
        x.stn.slave = eg[3] >> 16;
        x.stn.loopback = (eg[0] & EG_LOOPBACK) ? 1u : 0u;
        x.stn.addr = eg[4];
        x.stn.svc_addr = eg[5];
    }
}

// The IPv4 egress state of a packet the conntrack stage runs, packed by k_egress_pairs
// (which derives it from the record and the LB stage's scratch words anyway) into the
// packet's 64-B line of g.est (written whole: partial lines cost the writer a read):
// the stage then loads it with four 16-B loads instead of the 64-B record plus the
// scratch words behind data-dependent branches.
//   d0 skb4_pack(s)   d1 {w4, chk | ttl << 16 | flags << 24, ep | rev_nat << 16, slave}
//   d2 {tuple daddr, ct_state addr, ct_state svc_addr, 0}   d3 0
enum : uint32_t { ES_LOOPBACK = 1 };

__device__ __forceinline__ void eg4_pack(const Eg4 &x, uint32_t ep, uint4 *d)
{
    uint32_t w4, chk;
    d[0] = skb4_pack(x.s, w4, chk);
    d[1] = make_uint4(w4, chk | (x.s.ttl & 0xFFu) << 16 | (x.stn.loopback ? ES_LOOPBACK : 0u) << 24,
                      (ep & 0xFFFFu) | (x.stn.rev_nat & 0xFFFFu) << 16, x.stn.slave);
    d[2] = make_uint4(x.t.daddr, x.stn.addr, x.stn.svc_addr, 0u);
    d[3] = make_uint4(0u, 0u, 0u, 0u);
}

__device__ __forceinline__ void eg4_unpack(const uint4 *d, uint32_t stride, Eg4 &x, uint32_t &ep, uint32_t &fl)
{
    const uint4 d0 = d[0], d1 = d[1], d2 = d[2];
    x.s = skb4_unpack(d0, d1.x, d1.y & 0x3FFu, stride);
    x.s.ttl = (d1.y >> 16) & 0xFFu;
    fl = d1.y >> 24;
    ep = d1.z & 0xFFFFu;
    x.stn = CtState{d1.z >> 16, (fl & ES_LOOPBACK) ? 1u : 0u, d1.w, d2.y, d2.z, 0u};
    x.t.nexthdr = x.s.nexthdr;
    x.t.saddr = (fl & ES_LOOPBACK) ? d2.z : x.s.saddr;            // (a loopback skb carries IPV4_LOOPBACK)
    x.t.daddr = d2.x;
    x.t.dport = x.t.sport = 0;
}

struct Eg6 {
    Skb6 s;
    Tuple6 t;
    CtState stn;
};

__device__ __forceinline__ void eg6_state(const Rec6 &r, const uint32_t *eg, Eg6 &x)
{
    x.s = skb6_from(r);
    if (eg[0] & EG_SVC) {
#pragma unroll
        for (int j = 0; j < 4; ++j) x.s.daddr[j] = eg[12 + j];
        if (eg[0] & EG_DPORT_RW) x.s.h.p2 = eg[2] >> 16;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { x.t.daddr[j] = x.s.daddr[j]; x.t.saddr[j] = x.s.saddr[j]; }
    x.t.nexthdr = x.s.nexthdr;
    x.t.dport = x.t.sport = 0;
    x.stn = CtState{eg[3] & 0xFFFFu, 0, eg[3] >> 16, 0, 0, 0};
    if (!(eg[0] & EG_SVC)) x.stn = CtState{0, 0, 0, 0, 0, 0};
}

// The IPv6 egress state, packed the same way into the packet's line of g.est:
//   d0 saddr  d1 daddr (after lb6_xlate)  d2 {len, nexthdr | type << 8 | tflags << 16 |
//   l4off << 24, ports, chk | hoplimit << 16}  d3 {ep, the service stage's rev_nat | slave
//   << 16 (0 without a service), 0, 0}
__device__ __forceinline__ void eg6_pack(const Eg6 &x, uint32_t ep, uint32_t svc, uint4 *d)
{
    const Skb6 &s = x.s;
    d[0] = make_uint4(s.saddr[0], s.saddr[1], s.saddr[2], s.saddr[3]);
    d[1] = make_uint4(s.daddr[0], s.daddr[1], s.daddr[2], s.daddr[3]);
    d[2] = make_uint4(s.len, (s.nexthdr & 0xFFu) | (s.h.type & 0xFFu) << 8 | (s.h.tflags & 0xFFu) << 16 |
                                 ((uint32_t)s.l4off & 0xFFu) << 24,
                      (s.h.p0 & 0xFFFFu) | s.h.p2 << 16,
                      chk2(s.h.c1) | chk2(s.h.c14) << 2 | chk2(s.h.c4) << 4 | chk2(s.h.c2a) << 6 | chk2(s.h.c2b) << 8 |
                          (s.hoplimit & 0xFFu) << 16);
    d[3] = make_uint4(ep & 0xFFFFu, svc, 0u, 0u);
}

__device__ __forceinline__ void eg6_unpack(const uint4 *d, uint32_t stride, Eg6 &x, uint32_t &ep)
{
    const uint4 d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3];
    Skb6 &s = x.s;
    s.saddr[0] = d0.x; s.saddr[1] = d0.y; s.saddr[2] = d0.z; s.saddr[3] = d0.w;
    s.daddr[0] = d1.x; s.daddr[1] = d1.y; s.daddr[2] = d1.z; s.daddr[3] = d1.w;
    s.len = d2.x;
    s.nexthdr = d2.y & 0xFFu;
    s.l4off = (int)(d2.y >> 24);
    s.avail = stride;
    s.h.type = (d2.y >> 8) & 0xFFu;
    s.h.tflags = (d2.y >> 16) & 0xFFu;
    s.h.p0 = d2.z & 0xFFFFu;
    s.h.p2 = d2.z >> 16;
    s.h.c1 = unchk2(d2.w & 3u);
    s.h.c14 = unchk2((d2.w >> 2) & 3u);
    s.h.c4 = unchk2((d2.w >> 4) & 3u);
    s.h.c2a = unchk2((d2.w >> 6) & 3u);
    s.h.c2b = unchk2((d2.w >> 8) & 3u);
    s.hoplimit = (d2.w >> 16) & 0xFFu;
    ep = d3.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) { x.t.daddr[j] = s.daddr[j]; x.t.saddr[j] = s.saddr[j]; }
    x.t.nexthdr = s.nexthdr;
    x.t.dport = x.t.sport = 0;
    x.stn = CtState{d3.y & 0xFFFFu, 0, d3.y >> 16, 0, 0, 0};
}

// ================================================================== pairs -> components
// Every conntrack entry a packet can read outside the service set contains one of
// the address pairs unioned here (SURVEY.md §7 hard part 1).  The one entry it can
// write outside them, the NATed tuple of a service create (daddr = backend, saddr
// = backend), is a blind write: k_egress_nat merges it into the component only
// when some packet reads its pair, else its write is deferred to k_nat_apply, which
// resolves writers of one key last-writer-wins, as the sequential run does.
// one packet of k_egress_pairs: its record `rw` (loaded when `have`), its packed conntrack
// input state left in es[0..3] (zero for a packet that reaches no conntrack stage)
template <int NW>
__device__ __forceinline__ void pairs_one(const DpParams &p, const BatchDev &b, const GroupScratch &g, uint32_t i,
                                          const RecT<NW> &rw, bool have, uint4 *es)
{
    {
        uint32_t *egp = g.eg + (size_t)i * EG_WORDS;
        const uint4 *e4 = reinterpret_cast<const uint4 *>(egp);
        uint32_t eg[EG_WORDS];                                    // the scratch words, four wide loads
        const uint4 e0 = e4[0];
        eg[0] = e0.x; eg[1] = e0.y; eg[2] = e0.z; eg[3] = e0.w;
        if ((eg[0] & EG_STAGE) != STAGE_CT) { g.gslot[i] = NONE; g.ifx[i] = 0; return; }
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            const uint4 v = e4[k];
            eg[4 * k] = v.x; eg[4 * k + 1] = v.y; eg[4 * k + 2] = v.z; eg[4 * k + 3] = v.w;
        }
        g.ifx[i] = ((eg[0] & EG_V6) ? BIT_V6 : 0u) |
                   ((eg[0] & (EG_V6 | EG_SVC)) == EG_SVC && eg[4] ? BIT_NAT_CAND : 0u);
        const EpDev ep = G(p.eps)[eg[1] & 0xFFFFu];
        Acct na{0, 0};                                            // speculative probes are not accounted
        if (!(eg[0] & EG_V6)) {
            Rec r;
            if (have) r = rec_head(rw);
            else rec_load(r, b, i, 4);
            Eg4 x;
            eg4_state(r, eg, x);
            eg4_pack(x, eg[1], es);
            es[2].w = ep.seclabel;                                // (the stage's SECLABEL with uniform tables)
            const uint32_t S = x.t.saddr;
            const uint32_t P = group_node(g, pair_hash4(S, x.t.daddr, SALT_CT4));
            g.gslot[i] = P;
            // local delivery sees the packet after the service / loopback rewrites; that
            // pair is P itself unless a loopback rewrite changed it (its node is P's)
            const bool same = (x.s.saddr == S && x.s.daddr == x.t.daddr) || (x.s.saddr == x.t.daddr && x.s.daddr == S);
            if (!same) uf_union(g, P, group_node(g, pair_hash4(x.s.saddr, x.s.daddr, SALT_CT4)));
            uint32_t na4, np;                                     // a loopback NAT entry's reply rev-NAT target
            if (x.stn.addr && x.stn.loopback && revnat4(p, x.stn.rev_nat, na4, np, na))
                uf_union(g, P, group_node(g, pair_hash4(na4, S, SALT_CT4)));
            // the entry lookup 1 would hit today: a REPLY with rev-NAT rewrites the packet
            Tuple4 t1 = x.t;
            uint32_t seen;
            const bool l4ok = ct_l4<false>(t1, x.s.h, CT_EGRESS, seen) >= 0;
            eg[9] = port_sig(t1);                                 // the key signature of this packet's
            eg[10] = t1.nexthdr;                                  // create (and NAT) tuples
            egp[9] = eg[9];
            egp[10] = eg[10];
            if (l4ok && S == x.t.daddr)                           // self-pair egress lookup keys
                uf_union(g, P, group_node(g, self_hash(S, eg[9], t1.nexthdr)));
            if (x.s.saddr == x.s.daddr) {                         // self-pair keys of the delivery lookups
                Tuple4 ti;
                ti.nexthdr = x.s.nexthdr;
                ti.daddr = x.s.daddr;
                ti.saddr = x.s.saddr;
                ti.dport = ti.sport = 0;
                if (ct_l4<false>(ti, x.s.h, CT_INGRESS, seen) >= 0)
                    uf_union(g, P, group_node(g, self_hash(ti.saddr, port_sig(ti), ti.nexthdr)));
            }
            if (l4ok && ep.ct4.buckets) {
                uint32_t k[4];
                t1.key(k);
                const int64_t sl = dev_find<Ct4Spec, false>(ep.ct4, k, nullptr);   // (no CT writes here)
                if (sl >= 0) {
                    CtE e;
                    ct_load_hot<Ct4Spec>(ep.ct4, sl, e);
                    uint32_t na4, np;
                    if ((e.w[9] >> 16) && revnat4(p, e.w[9] >> 16, na4, np, na)) {
                        const bool lb = e.bits() & CTB_LB_LOOPBACK;
                        const uint32_t other = lb ? x.s.saddr : x.s.daddr;
                        uf_union(g, P, group_node(g, pair_hash4(na4, other, SALT_CT4)));
                        if (na4 == other)                         // a rewritten self pair: any ports
                            uf_union(g, P, group_node(g, self_hash(na4, 0, 0x100)));
                    }
                }
            }
        } else {
            Rec6 r;
            if constexpr (NW >= 32) {
                if (have) r = rw;
                else rec_load(r, b, i, 8);
            } else {
                rec_load(r, b, i, 8);                             // (a 64-B batch holds no IPv6 stage packet)
            }
            Eg6 x;
            eg6_state(r, eg, x);
            eg6_pack(x, eg[1], (eg[0] & EG_SVC) ? eg[3] : 0u, es);
            es[3].z = ep.seclabel;
            const uint32_t P = group_node(g, pair_hash6(x.t.saddr, x.t.daddr, SALT_CT6));
            g.gslot[i] = P;
            uint32_t xs[4] = {x.s.saddr[0], x.s.saddr[1], x.s.saddr[2], x.s.saddr[3]};
            Tuple6 t1 = x.t;
            uint32_t seen;
            if (x.s.l4off >= 0 && ct_l4<true>(t1, x.s.h, CT_EGRESS, seen) >= 0) {
                uint32_t k[10];
                t1.key(k);
                const int64_t sl = dev_find<Ct6Spec, false>(ep.ct6, k, nullptr);
                if (sl >= 0) {
                    CtE e;
                    ct_load_hot<Ct6Spec>(ep.ct6, sl, e);
                    uint32_t na6[4], np;
                    if ((e.w[9] >> 16) && revnat6(p, e.w[9] >> 16, na6, np, na)) {
                        uf_union(g, P, group_node(g, pair_hash6(na6, x.s.daddr, SALT_CT6)));
                        xs[0] = na6[0]; xs[1] = na6[1]; xs[2] = na6[2]; xs[3] = na6[3];
                    }
                }
            }
            // an entry the destination's ipv6_policy creates carries rev_nat_index =
            // low 16 bits of the destination address; a reply through it is rev-NATed
            uint32_t na6[4], np;
            if ((x.s.daddr[3] & 0xFFFFu) && revnat6(p, x.s.daddr[3] & 0xFFFFu, na6, np, na)) {
                uf_union(g, P, group_node(g, pair_hash6(na6, x.t.saddr, SALT_CT6)));
                uf_union(g, P, group_node(g, pair_hash6(na6, xs, SALT_CT6)));
            }
        }
    }
}

// The records come in through LDS (a wave's 64 consecutive records in coalesced 1-KiB
// loads) and the packed input states leave the same way, one 64-B line per packet.
template <int NW>
__global__ void __launch_bounds__(BLOCK) CV_WAVES_ATTR(CV_PAIRS_WAVES) k_egress_pairs(DpParams p, BatchDev b, GroupScratch g)
{
    __shared__ uint4 stage[BLOCK / 64][16 * NW];
    uint4 *st = stage[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < b.n; i0 += gridDim.x * BLOCK) {
        const uint32_t i = i0 + lane;
        const bool full = i0 + 64 <= b.n && b.stride == 4 * NW;  // (wave-uniform)
        RecT<NW> rw;
        if (full) rec_load_coop(rw, b, i0, st);
        uint4 es[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) es[k] = make_uint4(0u, 0u, 0u, 0u);
        if (i < b.n) pairs_one<NW>(p, b, g, i, rw, full, es);
        if (full) {
            wave_store64(g.est + (size_t)i0 * 4, es, st);
        } else if (i < b.n) {
#pragma unroll
            for (int k = 0; k < 4; ++k) g.est[(size_t)i * 4 + k] = es[k];
        }
    }
}

__global__ void __launch_bounds__(BLOCK) k_egress_nat(DpParams p, BatchDev b, GroupScratch g)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        if (!(g.ifx[i] & BIT_NAT_CAND)) continue;                // (STAGE_CT, IPv4 service, a NATed tuple)
        if (p.ct_guard) continue;                                 // one-packet launch: written inline, in order
        uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
        uint32_t nn;
        if (p.eg_left) {
            // admission: every writer joins the group of its NAT key's readers (a node
            // made if none reads it), so the writes run inline, in packet order, and
            // each draws on its packet's budget as the reference's create does
            if (eg[0] & EG_LOOPBACK) {
                nn = group_node(g, pair_hash4(eg[4], eg[5], SALT_CT4));
            } else {
                nn = group_node(g, self_hash(eg[4], eg[9], eg[10]));
                const uint32_t any = group_find(g, self_hash(eg[4], 0, 0x100));
                if (any != NONE) uf_union(g, g.gslot[i], any);
            }
        } else if (eg[0] & EG_LOOPBACK) {                         // (client, IPV4_LOOPBACK): by pair
            nn = group_find(g, pair_hash4(eg[4], eg[5], SALT_CT4));
        } else {                                                  // (backend, backend, ports, proto)
            nn = group_find(g, self_hash(eg[4], eg[9], eg[10]));
            if (nn == NONE) nn = group_find(g, self_hash(eg[4], 0, 0x100));
        }
        if (nn != NONE) {
            uf_union(g, g.gslot[i], nn);
        } else {
            eg[0] |= EG_NAT_DEFER;
            g.ifx[i] |= BIT_NAT_DEFER;
        }
    }
}

// Every packet of a conntrack stage keyed by its component (the union-find root of its
// address-pair node) for the binned grouping (k_gbin_group, flat lists: the groups'
// first packets in packet order, about the order the node-table queue used to have)
__global__ void __launch_bounds__(BLOCK) k_group_link(BatchDev b, GroupScratch g)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        const uint32_t s = g.gslot[i];
        g.hword[i] = 0;
        if (s == NONE) { g.pkey[i] = 0; continue; }
        const uint64_t root = uf_find(g, s);
        g.pkey[i] = (mix64(root ^ 0xC0FFEE0000000000ULL) & ~3ull) | 2ull | ((g.ifx[i] & BIT_V6) ? 1ull : 0ull);
    }
}

// ================================================================== egress conntrack + delivery
// The forwarded IPv4 frame of handle_ipv4_from_lxc: lb4_xlate (the LB stage's decision,
// from the scratch words), the egress reverse NAT, then ipv4_l3 of the exit taken
// (kind 0 pass_to_stack: dmac NODE_MAC; 1 to_host: NODE_MAC -> HOST_IFINDEX_MAC;
// 2 ipv4_local_delivery: the endpoint's node_mac -> mac) and the destination
// program's reverse NAT.
__device__ __noinline__ void eg4_frame(const DpParams &p, const BatchDev &b, const OutDev &o, const uint32_t *eg,
                                       uint32_t i, const EpDev &ep, const RevNatOut &rn1, int kind, int64_t lxc_slot,
                                       const RevNatOut &rn2)
{
    Rec r;
    rec_load(r, b, i, 3);
    const uint8_t *in = b.frames + (size_t)i * b.stride;
    Frame4 f;
    frame4_init(f, r, in);
    if (eg[0] & EG_SVC)
        frame4_xlate(f, f.daddr, eg[7], (eg[0] & EG_LOOPBACK) ? eg[8] : 0u, eg[0] & EG_DPORT_RW, eg[2] & 0xFFFFu,
                     eg[2] >> 16);
    if (rn1.valid) frame4_revnat(f, rn1.na, rn1.np, rn1.loopback, f.saddr);
    if (kind == 0) {
        frame4_l3(f, nullptr, ep.node_mac);
    } else if (kind == 1) {
        frame4_l3(f, ep.node_mac, p.host_mac);
    } else {
        uint32_t mac[2], nmac[2];
        lxc_macs(p.lxc4, lxc_slot, mac, nmac);
        frame4_l3(f, nmac, mac);
        if (rn2.valid) frame4_revnat(f, rn2.na, rn2.np, false, f.saddr);
    }
    frame4_emit(f, in, o.frames + (size_t)i * b.stride, b.stride, r.len);
}

template <bool Q, class M>
__device__ __forceinline__ void deliver4_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                             const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq);
template <bool Q, class M>
__device__ __forceinline__ void deliver6_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                             const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq);

// handle_ipv4_from_lxc (bpf_lxc.c:464-649) from skip_service_lookup on.  INL: the local
// delivery runs inline (the continuation list, whose lanes run several members of a
// group in one launch), else it is handed to k_egress_deliver.  Q: every lane of the
// wave calls (live = false: no packet), so the ipcache, policy and endpoint lookups are
// quad probes at convergent call sites; `state` replaces the early exits: 0 going on,
// 1 final (outputs written), 2 dropped with `ret`.
template <bool INL, bool Q, class M>
__device__ __forceinline__ void egress4_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                            const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq)
{
    const uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
    Eg4 x{};
    uint32_t epi = 0, fl = 0;
    EpDev ep{};
    Acct a{0, 0, m.pc};
    a.ctu = ct_unit(p);
    if (live) {
        eg4_unpack(g.est + (size_t)i * 4, b.stride, x, epi, fl);
        // the source endpoint's tables and SECLABEL from its EpHot line (with one policy
        // and CT4 map for every endpoint: the common line, SECLABEL from the state); the
        // full EpDev where the event records need its constants
        ep = ep_netdev4<M::EV>(p, epi);
        if (!M::EV) ep.seclabel = g.est[(size_t)i * 4 + 2].w;
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        m.src_id = ep.lxc_id;
        m.src_label = ep.seclabel;
        a.nl = o.nl ? o.nl[i] : 0u;
        a.nu = o.nu ? o.nu[i] : 0u;
    }
    EgAdm adm(p, i, a, live, M::SN);
    EgOut res{TC_ACT_OK, 0, 0, CT_NONE, 0};
    Skb4 &s = x.s;
    Tuple4 &t = x.t;
    CtState st{0, 0, 0, 0, 0, 0};
    int64_t slot = -1;
    const uint32_t orig_dip = t.daddr;
    bool mon = false;
    int ret = live ? ct_lookup<false, EGF>(ep.ct4, t, s.h, CT_EGRESS, s.len, now, p.flags, slot, &st, a, &mon) : 0;
    int state = !live ? 1 : ret < 0 ? 2 : 0;
    RevNatOut rn1{false, false, 0, 0}, rn2{false, false, 0, 0};   // reverse NATs applied (output frames)
    // destination category (:482-494): the ipcache identity of the original daddr
    const uint32_t lab = ipcache4_at<Q>(p, orig_dip, state == 0, a, sq);
    if (state == 0) {
        res.ct = (uint8_t)ret;
        res.dst = lab ? lab : ((orig_dip & p.v4_cluster_mask) == p.v4_cluster_range ? CLUSTER_ID : WORLD_ID);
    }
    const int verdict = policy_egress_at<Q>(ep.policy, p.flags, s.len, res.dst, t.dport, t.nexthdr, a, state == 0, sq);
    if (state == 0) {
        if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
            if (ret == CT_ESTABLISHED) {
                ct_kill<Ct4Spec>(ep.ct4, slot, a, p.ct_guard);   // ct_delete4
                eg_changed();
            }
            ret = verdict;
            state = 2;
        } else if (ret == CT_NEW) {
            x.stn.src_sec_id = ep.seclabel;
            const bool defer = g.ifx[i] & BIT_NAT_DEFER;
            const int c = ct_create<false>(ep.ct4, t, s.len, CT_EGRESS, x.stn, now, a, p.ct_guard, defer, true);
            eg_changed();
            if (defer && c != DROP_CT_CREATE_FAILED) g.ifx[i] |= BIT_NAT_DONE;
            if (is_err(c)) { ret = c; state = 2; }
        } else if ((ret == CT_REPLY || ret == CT_RELATED) && st.rev_nat) {   // lb4_rev_nat(.., 0)
            uint32_t na, np;
            if (revnat4(p, st.rev_nat, na, np, a)) {
                const int r2 = rev_map_port(s.h, t.nexthdr, np);
                const int r3 = r2 ? 0 : l4_csum_err(s, t.nexthdr);   // __lb4_rev_nat checksum updates
                if (r2 || r3) {
                    ret = r2 ? r2 : r3;
                    state = 2;
                } else {
                    rn1 = RevNatOut{true, st.loopback != 0, na, np};
                    const uint32_t old_sip = s.saddr;
                    if (st.loopback) s.daddr = old_sip;
                    s.saddr = na;
                }
            }
        }
        if (state == 0 && verdict > 0) {                          // ipv4_redirect_to_host_port + ipv4_l3
            notify_trace(p, m, TRACE_TO_PROXY, s.len, ep.lxc_id, ep.seclabel, 0, 0, HOST_IFINDEX, res.ct, mon);
            res.proxy = (uint16_t)verdict;
            if (s.ttl <= 1) {
                ret = DROP_INVALID;
                state = 2;
            } else {
                res.ret = TC_ACT_REDIRECT;
                eg_done(g, i, res, a);
                state = 1;
            }
        }
    }
    uint32_t iv = 0;                                              // lookup_ip4_endpoint(ip4)
    int64_t lxc_slot = -1;
    if (p.lxc4.buckets) {
        if (state == 0) a.nl++;
        lxc_slot = find_q<Q, LxcV4Spec>(p.lxc4, &s.daddr, state == 0, sq, &iv);
    }
    if (state == 0) {
        if (s.ttl <= 1) {                                         // ipv4_l3 -> ipv4_dec_ttl
            ret = DROP_INVALID;
            state = 2;
        } else if (lxc_slot >= 0) {
            m.fwd(s.len, METRIC_EGRESS);                          // TRACE_TO_HOST / ipv4_local_delivery
            const uint32_t e2 = (iv & (1u << 16)) ? 0u : p.ep_of_lxc ? p.ep_of_lxc[iv & 0xFFFFu] : 0u;
            if (iv & (1u << 16)) {                                // to_host
                res.ret = TC_ACT_REDIRECT;
                notify_trace(p, m, TRACE_TO_HOST, s.len, ep.lxc_id, ep.seclabel, HOST_ID, 0, HOST_IFINDEX, res.ct, mon);
                if (M::EV && o.frames) eg4_frame(p, b, o, eg, i, ep, rn1, 1, -1, rn2);
                eg_done(g, i, res, a);
            } else if (!e2) {
                ret = DROP_MISSED_TAIL_CALL;
                state = 2;
            } else {
                // ipv4_local_delivery -> the destination's handle_policy: k_egress_deliver,
                // or (split) the record handed over to the destination's rank
                uint32_t w4, chk;
                uint4 *d = (o.deliver ? o.deliver : g.del) + (size_t)i * DEL_SLOTS;
                d[0] = skb4_pack(s, w4, chk);
                d[1] = make_uint4(w4, chk | (a.nl & 0xFFu) << 16 | (a.nu & 0xFFu) << 24,
                                  (e2 - 1) | (uint32_t)res.ct << 16 | (rn1.valid ? 1u << 25 : 0u) |
                                      (rn1.loopback ? 1u << 26 : 0u),
                                  ep.seclabel);
                d[2] = make_uint4(ifindex_of(m, p.lxc4, lxc_slot, iv), res.dst, (uint32_t)lxc_slot, rn1.na);
                if (M::EV) g.del_ev[2 * (size_t)i] = make_uint4(rn1.np, 0, 0, 0);
                if (o.deliver) {
                    d[3] = make_uint4(0u, 0u, 0u, 0u);
                    res.ret = E_DEFER;
                    eg_done(g, i, res, a);
                } else {
                    adm.flush();                                  // (the delivery draws on what is left)
                    if constexpr (INL) deliver4_one<false>(p, b, now, o, g, i, true, m, sq);
                    else del_list(g, false, i);
                }
            }
        } else {                                                  // pass_to_stack: ipv4_l3
            m.fwd(s.len, METRIC_EGRESS);                          // TRACE_TO_STACK
            notify_trace(p, m, TRACE_TO_STACK, s.len, ep.lxc_id, ep.seclabel, res.dst, 0, 0, res.ct, mon);
            res.ret = TC_ACT_OK;
            if (M::EV && o.frames) eg4_frame(p, b, o, eg, i, ep, rn1, 0, -1, rn2);
            eg_done(g, i, res, a);
        }
    }
    if (state == 2) {
        eg_drop(p, res, ret, s.len, m);
        eg_done(g, i, res, a);
    }
}

// The forwarded IPv6 frame of ipv6_l3_from_lxc: lb6_xlate (the LB stage's target and
// port from the scratch words), the egress reverse NAT, then ipv6_l3 of the exit taken
// (kind 0 pass_to_stack: dmac NODE_MAC + ipv6_store_flowlabel; 1 to_host: NODE_MAC ->
// HOST_IFINDEX_MAC; 2 ipv6_local_delivery: the endpoint's node_mac -> mac, then the
// destination's ipv6_policy: rev-NAT index zeroing and reverse NAT).
__device__ __noinline__ void eg6_frame(const DpParams &p, const BatchDev &b, const OutDev &o, const uint32_t *eg,
                                       uint32_t i, const EpDev &ep, const RevNat6Out &rn1, int kind, int64_t lxc_slot,
                                       const RevNat6Out &rn2)
{
    Rec6 r;
    rec_load(r, b, i, 8);
    const uint8_t *in = b.frames + (size_t)i * b.stride;
    uint32_t nh = rec_u8c<20>(r);
    const int hl = ipv6_hdrlen(r, nh);
    Frame6 f;
    frame6_init(f, r, hl < 0 ? hl : 14 + hl, nh, in);
    if (eg[0] & EG_SVC) frame6_xlate(f, eg + 12, eg[0] & EG_DPORT_RW, eg[2] & 0xFFFFu, eg[2] >> 16);
    if (rn1.valid) frame6_revnat(f, rn1);
    if (kind == 0) {
        frame6_l3(f, nullptr, ep.node_mac);
        frame6_flowlabel(f, ep.seclabel);
    } else if (kind == 1) {
        frame6_l3(f, ep.node_mac, p.host_mac);
    } else {
        uint32_t mac[2], nmac[2];
        lxc_macs(p.lxc6, lxc_slot, mac, nmac);
        frame6_l3(f, nmac, mac);
        frame6_zero_revnat(f);
        if (rn2.valid) frame6_revnat(f, rn2);
    }
    frame6_emit(f, in, o.frames + (size_t)i * b.stride, b.stride);
}

// ipv6_l3_from_lxc (bpf_lxc.c:133-352) from skip_service_lookup on; Q / live / state as
// egress4_one (here the policy lookup is the quad probe: the IPv6 endpoint and ipcache
// tables have 128-B buckets, probed tag-first per lane)
template <bool INL, bool Q, class M>
__device__ __forceinline__ void egress6_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                            const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq)
{
    const uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
    Eg6 x{};
    uint32_t epi = 0;
    EpDev ep{};
    Acct a{0, 0, m.pc};
    a.ctu = ct_unit(p);
    if (live) {
        eg6_unpack(g.est + (size_t)i * 4, b.stride, x, epi);
        ep = ep_uni6<M::EV>(p, epi);
        if (!M::EV) ep.seclabel = g.est[(size_t)i * 4 + 3].z;
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        m.src_id = ep.lxc_id;
        m.src_label = ep.seclabel;
        a.nl = o.nl ? o.nl[i] : 0u;
        a.nu = o.nu ? o.nu[i] : 0u;
    }
    EgAdm adm(p, i, a, live, M::SN);
    EgOut res{TC_ACT_OK, 0, 0, CT_NONE, 0};
    Skb6 &s = x.s;
    Tuple6 &t = x.t;
    CtState st{0, 0, 0, 0, 0, 0};
    int64_t slot = -1;
    const uint32_t orig_dip[4] = {t.daddr[0], t.daddr[1], t.daddr[2], t.daddr[3]};
    bool mon = false;
    int ret = live ? ct_lookup<true, EGF, true>(ep.ct6, t, s.h, CT_EGRESS, s.len, now, p.flags, slot, &st, a, &mon) : 0;
    int state = !live ? 1 : ret < 0 ? 2 : 0;
    RevNat6Out rn1, rn2;                                          // reverse NATs applied (output frames)
    rn1.valid = rn2.valid = false;
    if (state == 0) {
        res.ct = (uint8_t)ret;
        const uint32_t lab = ipcache6(p, orig_dip, a);
        res.dst = lab ? lab
                      : ((s.daddr[0] == p.router6[0] && s.daddr[1] == p.router6[1]) ? CLUSTER_ID : WORLD_ID);
    }
    const int verdict = policy_egress_at<Q>(ep.policy, p.flags, s.len, res.dst, t.dport, t.nexthdr, a, state == 0, sq);
    if (state == 0) {
        if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
            if (ret == CT_ESTABLISHED) {
                ct_kill<Ct6Spec>(ep.ct6, slot, a, p.ct_guard);   // ct_delete6
                eg_changed();
            }
            ret = verdict;
            state = 2;
        } else if (ret == CT_NEW) {
            x.stn.src_sec_id = ep.seclabel;
            const int c = ct_create<true>(ep.ct6, t, s.len, CT_EGRESS, x.stn, now, a, p.ct_guard, false, true);
            eg_changed();
            if (is_err(c)) { ret = c; state = 2; }
        } else if ((ret == CT_REPLY || ret == CT_RELATED) && st.rev_nat) {   // lb6_rev_nat(.., 0)
            uint32_t na[4], np;
            if (revnat6(p, st.rev_nat, na, np, a)) {
                const int r2 = rev_map_port(s.h, t.nexthdr, np);
                const int r3 = r2 ? 0 : l4_csum_err6(s);          // __lb6_rev_nat checksum update
                if (r2 || r3) {
                    ret = r2 ? r2 : r3;
                    state = 2;
                } else {
                    rn1.valid = true;
                    rn1.np = np;
#pragma unroll
                    for (int j = 0; j < 4; ++j) { s.saddr[j] = na[j]; rn1.na[j] = na[j]; }
                }
            }
        }
        if (state == 0 && verdict > 0) {                          // ipv6_redirect_to_host_port + ipv6_l3
            notify_trace(p, m, TRACE_TO_PROXY, s.len, ep.lxc_id, ep.seclabel, 0, 0, HOST_IFINDEX, res.ct, mon);
            res.proxy = (uint16_t)verdict;
            if (s.hoplimit <= 1) {
                ret = E_PUNT;
                state = 2;
            } else {
                res.ret = TC_ACT_REDIRECT;
                eg_done(g, i, res, a);
                state = 1;
            }
        }
    }
    if (state == 0) {
        uint32_t iv = 0;
        int64_t lxc_slot = -1;
        if (p.lxc6.buckets) {                                     // lookup_ip6_endpoint (the daddr is unchanged)
            a.nl++;
            lxc_slot = dev_find<LxcV6Spec>(p.lxc6, s.daddr, &iv);
        }
        if (s.hoplimit <= 1) {                                    // icmp6_send_time_exceeded / ipv6_l3
            ret = E_PUNT;
            state = 2;
        } else if (lxc_slot >= 0) {
            m.fwd(s.len, METRIC_EGRESS);
            const uint32_t e2 = (iv & (1u << 16)) ? 0u : p.ep_of_lxc ? p.ep_of_lxc[iv & 0xFFFFu] : 0u;
            if (iv & (1u << 16)) {                                // to_host
                res.ret = TC_ACT_REDIRECT;
                notify_trace(p, m, TRACE_TO_HOST, s.len, ep.lxc_id, ep.seclabel, HOST_ID, 0, HOST_IFINDEX, res.ct, mon);
                if (M::EV && o.frames) eg6_frame(p, b, o, eg, i, ep, rn1, 1, -1, rn2);
                eg_done(g, i, res, a);
            } else if (!e2) {
                ret = DROP_MISSED_TAIL_CALL;
                state = 2;
            } else {
                // ipv6_local_delivery -> the destination's handle_policy: k_egress_deliver,
                // or (split) the record handed over to the destination's rank
                uint4 *d = (o.deliver ? o.deliver : g.del) + (size_t)i * DEL_SLOTS;
                d[0] = make_uint4(s.saddr[0], s.saddr[1], s.saddr[2], s.saddr[3]);
                d[1] = make_uint4(s.daddr[0], s.daddr[1], s.daddr[2], s.daddr[3]);
                d[2] = make_uint4(s.len, (s.nexthdr & 0xFFu) | (s.h.type & 0xFFu) << 8 | (s.h.tflags & 0xFFu) << 16 |
                                             ((uint32_t)s.l4off & 0xFFu) << 24,
                                  (s.h.p0 & 0xFFFFu) | s.h.p2 << 16,
                                  chk2(s.h.c1) | chk2(s.h.c14) << 2 | chk2(s.h.c4) << 4 | chk2(s.h.c2a) << 6 |
                                      chk2(s.h.c2b) << 8 | (a.nl & 0xFFu) << 16 | (a.nu & 0xFFu) << 24);
                d[3] = make_uint4((e2 - 1) | (uint32_t)res.ct << 16 | (rn1.valid ? 1u << 25 : 0u), ep.seclabel,
                                  ifindex_of(m, p.lxc6, lxc_slot, iv), res.dst);
                if (M::EV) {
                    g.del_ev[2 * (size_t)i] = make_uint4((uint32_t)lxc_slot, rn1.np, 0, 0);
                    g.del_ev[2 * (size_t)i + 1] = make_uint4(rn1.na[0], rn1.na[1], rn1.na[2], rn1.na[3]);
                }
                if (o.deliver) {
                    res.ret = E_DEFER;
                    eg_done(g, i, res, a);
                } else {
                    adm.flush();
                    if constexpr (INL) deliver6_one<false>(p, b, now, o, g, i, true, m, sq);
                    else del_list(g, true, i);
                }
            }
        } else {
            m.fwd(s.len, METRIC_EGRESS);
            notify_trace(p, m, TRACE_TO_STACK, s.len, ep.lxc_id, ep.seclabel, res.dst, 0, 0, res.ct, mon);
            res.ret = TC_ACT_OK;
            if (M::EV && o.frames) eg6_frame(p, b, o, eg, i, ep, rn1, 0, -1, rn2);
            eg_done(g, i, res, a);
        }
    }
    if (state == 2) {
        eg_drop(p, res, ret, s.len, m);
        eg_done(g, i, res, a);
    }
}

// ================================================================== local delivery
// A packet k_egress_ct forwards to a local endpoint leaves its state after the egress
// program in a delivery record (g.del) and joins the position's delivery list; the
// destination's policy program (handle_policy -> ipv{4,6}_policy) runs for the whole
// list in k_egress_deliver, right after the k_egress_ct launch of the same position.
// The packets of one position belong to different groups (no common conntrack entry),
// so running all their egress halves before all their delivery halves equals running
// each packet whole; the next position's launch follows both.  The split keeps the
// delivery path out of the egress kernel's registers (it spilled over a hundred VGPRs
// to scratch) and runs the deliveries with every lane on the same path.
template <bool Q, class M>
__device__ __forceinline__ void deliver4_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                             const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq)
{
    uint4 d0{}, d1{}, d2{};
    if (live) {
        const uint4 *d = g.del + (size_t)i * DEL_SLOTS;
        d0 = d[0]; d1 = d[1]; d2 = d[2];
    }
    Skb4 s = skb4_unpack(d0, d1.x, d1.y & 0x3FFu, b.stride);
    Acct a{(d1.y >> 16) & 0xFFu, d1.y >> 24, m.pc};
    a.ctu = ct_unit(p);
    EgAdm adm(p, i, a, live, M::SN, 1, d1.z & 0xFFFFu);
    EgOut res{TC_ACT_OK, 0, d2.y, (uint8_t)(d1.z >> 16), 0};
    if (live) {
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
    }
    RevNatOut rn2{false, false, 0, 0};
    uint8_t ct2 = CT_NONE;
    // the destination's tables from its EpHot line (the full EpDev for the event records)
    const EpDev ep = live ? ep_netdev4<M::EV>(p, d1.z & 0xFFFFu) : EpDev{};
    res.ret = handle_policy4<M, EGF, Q>(p, ep, s, d1.w, false, d2.x, now, ct2, res.proxy, res.reason, a, m, &rn2,
                                        nullptr, live, sq);
    if (!live) return;
    if (M::EV && o.frames && (res.ret == TC_ACT_OK || res.ret == TC_ACT_REDIRECT) && !res.proxy) {
        const uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
        const RevNatOut rn1{(d1.z >> 25) & 1u ? true : false, (d1.z >> 26) & 1u ? true : false, d2.w,
                            g.del_ev[2 * (size_t)i].x};
        eg4_frame(p, b, o, eg, i, G(p.eps)[eg[1] & 0xFFFFu], rn1, 2, (int64_t)d2.z, rn2);   // ipv4_local_delivery
    }
    eg_done(g, i, res, a);
}

template <bool Q, class M>
__device__ __forceinline__ void deliver6_one(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                             const GroupScratch &g, uint32_t i, bool live, M &m, uint4 *sq)
{
    uint4 d0{}, d1{}, d2{}, d3{};
    if (live) {
        const uint4 *d = g.del + (size_t)i * DEL_SLOTS;
        d0 = d[0]; d1 = d[1]; d2 = d[2]; d3 = d[3];
    }
    Skb6 s;
    s.saddr[0] = d0.x; s.saddr[1] = d0.y; s.saddr[2] = d0.z; s.saddr[3] = d0.w;
    s.daddr[0] = d1.x; s.daddr[1] = d1.y; s.daddr[2] = d1.z; s.daddr[3] = d1.w;
    s.len = d2.x;
    s.nexthdr = d2.y & 0xFFu;
    s.hoplimit = 0;                                               // (checked before the hand-over)
    s.l4off = (int)(d2.y >> 24);
    s.avail = b.stride;
    s.h.type = (d2.y >> 8) & 0xFFu;
    s.h.tflags = (d2.y >> 16) & 0xFFu;
    s.h.p0 = d2.z & 0xFFFFu;
    s.h.p2 = d2.z >> 16;
    s.h.c1 = unchk2(d2.w & 3u);
    s.h.c14 = unchk2((d2.w >> 2) & 3u);
    s.h.c4 = unchk2((d2.w >> 4) & 3u);
    s.h.c2a = unchk2((d2.w >> 6) & 3u);
    s.h.c2b = unchk2((d2.w >> 8) & 3u);
    Acct a{(d2.w >> 16) & 0xFFu, d2.w >> 24, m.pc};
    a.ctu = ct_unit(p);
    EgAdm adm(p, i, a, live, M::SN, 1, d3.x & 0xFFFFu);
    EgOut res{TC_ACT_OK, 0, d3.w, (uint8_t)(d3.x >> 16), 0};
    if (live) {
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
    }
    RevNat6Out rn2;
    rn2.valid = false;
    uint8_t ct2 = CT_NONE;
    const EpDev ep = live ? ep_uni6<M::EV>(p, d3.x & 0xFFFFu) : EpDev{};
    res.ret = handle_policy6<M, EGF, Q>(p, ep, s, d3.y, false, d3.z, now, ct2, res.proxy, res.reason, a, m, &rn2,
                                        nullptr, live, sq);
    if (!live) return;
    if (M::EV && o.frames && (res.ret == TC_ACT_OK || res.ret == TC_ACT_REDIRECT) && !res.proxy) {
        const uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
        const uint4 d4 = g.del_ev[2 * (size_t)i], d5 = g.del_ev[2 * (size_t)i + 1];
        RevNat6Out rn1;
        rn1.valid = (d3.x >> 25) & 1u;
        rn1.np = d4.y;
        rn1.na[0] = d5.x; rn1.na[1] = d5.y; rn1.na[2] = d5.z; rn1.na[3] = d5.w;
        eg6_frame(p, b, o, eg, i, G(p.eps)[eg[1] & 0xFFFFu], rn1, 2, (int64_t)d4.x, rn2);   // ipv6_local_delivery
    }
    eg_done(g, i, res, a);
}

// the wave-uniform loop over the list of the deliveries a position handed over: every
// lane of a wave calls fn the same number of times (live = false past the end)
template <class F>
__device__ __forceinline__ void for_each_wave(uint32_t total, F &&fn)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t j0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); j0 < total; j0 += stride) {
        const uint32_t j = j0 + lane;
        fn(j, j < total);
    }
}

// Occupancy of the egress conntrack stage: left alone the compiler spends 177 VGPRs
// (2 waves/SIMD) on a lane whose time goes to ~15-20 dependent memory round trips;
// capping it at 4 waves/SIMD (<= 128 VGPRs) hides more of that latency: config 5
// 880 -> 971 Mpps (A/B on the box: 3 waves 958, 5 waves 809)
#ifndef CV_EG_WAVES
#define CV_EG_WAVES 4
#endif
#define CV_EG_OCC __attribute__((amdgpu_waves_per_eu(CV_EG_WAVES, 8)))

template <bool V6, bool EV, bool SN = false>
__global__ void __launch_bounds__(BLOCK) CV_EG_OCC k_egress_deliver(DpParams p, BatchDev b, uint32_t now, OutDev o,
                                                                     GroupScratch g)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    __shared__ uint4 stage[BLOCK / 64][256];                      // quad probes
    uint4 *sq = stage[threadIdx.x >> 6];
    using M = MetT<EV, SN>;
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    const uint32_t total = g.cursor[del_ctr(V6, g.pos)];
    for_each_wave(total, [&](uint32_t j, bool live) {
        uint32_t i = live ? g.single[j] : 0u;
        if (live && !pkt_ok(g, i)) { live = false; i = 0u; }
        if constexpr (V6) deliver6_one<true>(p, b, now, o, g, i, live, m, sq);
        else deliver4_one<true>(p, b, now, o, g, i, live, m, sq);
    });
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}


// the continuation list's instance takes a budget of its own (its lanes walk several
// members of a group and deliver inline: more live state per lane; at 4 waves / SIMD it
// spilled 48-64 B per lane).  A/B on one box, two runs each (`profiles/r06g`): 4 waves
// 3.51 ms per step, 3 waves 3.36, 2 waves 3.38 -- config 5 1 273 -> 1 291 Mpps
#ifndef CV_EG_CONT_WAVES
#define CV_EG_CONT_WAVES 3
#endif
#define CV_EG_CONT_OCC __attribute__((amdgpu_waves_per_eu(CV_EG_CONT_WAVES, 8)))

template <bool V6, bool EV, bool INL, bool SN>
__device__ __forceinline__ void egress_ct_body(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                               const GroupScratch &g, uint32_t pos);

template <bool V6, bool EV, bool INL, bool SN = false>
__global__ void __launch_bounds__(BLOCK) CV_EG_OCC k_egress_ct(DpParams p, BatchDev b, uint32_t now, OutDev o, GroupScratch g,
                                                                uint32_t pos)
{
    egress_ct_body<V6, EV, INL, SN>(p, b, now, o, g, pos);
}

template <bool V6, bool EV, bool SN = false>
__global__ void __launch_bounds__(BLOCK) CV_EG_CONT_OCC k_egress_cont(DpParams p, BatchDev b, uint32_t now, OutDev o,
                                                                       GroupScratch g, uint32_t pos)
{
    egress_ct_body<V6, EV, true, SN>(p, b, now, o, g, pos);
}

template <bool V6, bool EV, bool INL, bool SN>
__device__ __forceinline__ void egress_ct_body(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o,
                                               const GroupScratch &g, uint32_t pos)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    __shared__ uint4 stage[BLOCK / 64][256];                      // quad probes
    uint4 *sq = stage[threadIdx.x >> 6];
    using M = MetT<EV, SN>;
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    const int q = V6 ? Q_CT6 : Q_CT4;
    if constexpr (INL) {
        // the continuation list: a lane runs the members of its group from `pos` on, lane
        // by lane (per-lane probes)
        for_each_at(g, q, pos, [&](uint32_t x) {
            if constexpr (V6) egress6_one<true, false>(p, b, now, o, g, x, true, m, sq);
            else egress4_one<true, false>(p, b, now, o, g, x, true, m, sq);
        });
    } else {
        // member `pos` of every group, in packet order (one launch per position); every
        // lane of a wave at the same call sites (quad probes)
        uint32_t base = 0;
        for (uint32_t l = 0; l < pos; ++l) base += g.cursor[qcls(q, l)];
        for_each_wave(g.cursor[qcls(q, pos)], [&](uint32_t j, bool live) {
            uint32_t x = live ? g.work[base + j] : 0u;
            if (live && !pkt_ok(g, x)) { live = false; x = 0u; }
            if constexpr (V6) egress6_one<false, true>(p, b, now, o, g, x, live, m, sq);
            else egress4_one<false, true>(p, b, now, o, g, x, live, m, sq);
        });
    }
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// ================================================================== deferred NAT tuples
// Writers of one NAT pair join one group; its lane writes each member's entry if
// no later packet of the launch wrote that key before (the padding words 14/15 of
// the 64-B value slot hold {epoch, writer}), so every key ends with the value of
// its highest-index writer.
__global__ void __launch_bounds__(BLOCK) k_nat_group(BatchDev b, GroupScratch g)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        if (!(g.ifx[i] & BIT_NAT_DONE)) { g.gslot[i] = NONE; continue; }
        const uint32_t *eg = g.eg + (size_t)i * EG_WORDS;
        group_push(g, group_node(g, pair_hash4(eg[4], eg[6], SALT_NAT)), i, Q_NAT);
    }
}

__global__ void __launch_bounds__(BLOCK) k_nat_apply(DpParams p, BatchDev b, uint32_t now, GroupScratch g)
{
    __shared__ LdsPolicy pc;                                      // the CT maps' live counts
    pol_cache_init(pc);
    __syncthreads();
    for_each_group(g, Q_NAT, [&](uint32_t, uint32_t head) {
        for (uint32_t x = head; x != NONE; x = g.next[x]) {
            Rec r;
            rec_load(r, b, x, 4);
            const uint32_t *eg = g.eg + (size_t)x * EG_WORDS;
            const EpDev ep = G(p.eps)[eg[1] & 0xFFFFu];
            Eg4 y;
            eg4_state(r, eg, y);
            uint32_t seen;
            ct_l4<false>(y.t, y.s.h, CT_EGRESS, seen);            // the tuple ct_create4 saw: reversed,
            y.t.reverse();                                        // after a NEW lookup
            y.stn.src_sec_id = ep.seclabel;
            CtE e;
            ct_entry_new(e, y.t.nexthdr == 6, y.s.len, CT_EGRESS, y.stn, now);
            const Tuple4 n = ct_nat_tuple(y.t, CT_EGRESS, y.stn);
            uint32_t k[4];
            n.key(k);
            bool created;
            const int64_t sl = dev_upsert<Ct4Spec>(ep.ct4, k, &created);
            if (sl < 0) continue;                                 // (probe limit; launches are planned with room)
            if (created && ep.ct4.live) live_add(&pc, ep.ct4.live, 1ull);
            const CV_G uint32_t *v = ct_cold<Ct4Spec>(ep.ct4, sl);  // w14 / w15: side words 4 / 5
            if (!created && v[5] == g.serial && v[4] > x) continue;
            e.w[14] = x;
            e.w[15] = g.serial;
            ct_store<Ct4Spec>(ep.ct4, sl, e, created);
        }
    });
    __syncthreads();
    pol_cache_flush(pc);
}

// ================================================================== delivery records
// cv_lxc_deliver: the destination's policy program (handle_policy -> ipv4_policy /
// ipv6_policy) of delivery records a source program left on another rank (endpoint-owned
// conntrack across GPUs).  Every entry the program reads or writes carries
// the record's address pair in the destination's CT map, so the records are grouped by
// (map, pair) with the binned grouping, each group in record order on one lane.
constexpr uint64_t SALT_DELIVER6 = 0x44454C3600000000ULL;
template <bool V6>
__global__ void __launch_bounds__(BLOCK) k_deliver_keys(DpParams p, BatchDev b, GroupScratch g)
{
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        const uint4 *d = g.del + (size_t)i * DEL_SLOTS;
        uint64_t gh = 0;
        uint32_t e;
        if constexpr (V6) {
            const uint4 d0 = d[0], d1 = d[1];
            e = d[3].x & 0xFFFFu;
            const uint32_t sa[4] = {d0.x, d0.y, d0.z, d0.w}, da[4] = {d1.x, d1.y, d1.z, d1.w};
            if (e < p.n_eps) gh = pair_hash6(sa, da, SALT_DELIVER6 ^ (uint64_t)(uintptr_t)G(p.eps)[e].ct6.buckets);
        } else {
            const uint4 d0 = d[0], d1 = d[1];
            e = d1.z & 0xFFFFu;
            const Skb4 s = skb4_unpack(d0, d1.x, d1.y & 0x3FFu, b.stride);
            if (e < p.n_eps) gh = pair_hash4(s.saddr, s.daddr, (uint64_t)(G(p.ephot)[e].ct_v4 & EPH_CT_ID) << 17);
        }
        if (e >= p.n_eps) group_err(g, GERR_INDEX);               // (a corrupt record: no program)
        g.pkey[i] = e < p.n_eps ? ((gh & ~3ull) | 2ull | (V6 ? 1ull : 0ull)) : 0ull;
        g.hword[i] = 0;
        g.gslot[i] = NONE;
        g.res[i] = make_uint4(0u, 0u, 0u, 0u);
    }
}

template <bool V6, bool SN = false>
__global__ void __launch_bounds__(BLOCK) k_deliver_runs(DpParams p, BatchDev b, uint32_t now, OutDev o, GroupScratch g)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    using M = MetT<false, SN>;                                    // (SN: admitted next to max_entries)
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    for_each_run(g, V6 ? Q_NETDEV6 : Q_NETDEV, false, [&](uint32_t x, uint32_t) {
        if constexpr (V6) deliver6_one<false>(p, b, now, o, g, x, true, m, nullptr);
        else deliver4_one<false>(p, b, now, o, g, x, true, m, nullptr);
    });
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

int launch_lxc_deliver(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o, GroupScratch g, int v6,
                       hipStream_t s)
{
    g.lim = b.n;
    if (!b.n) return 0;
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    if (v6) hipLaunchKernelGGL(k_deliver_keys<true>, grid, blk, 0, s, p, b, g);
    else hipLaunchKernelGGL(k_deliver_keys<false>, grid, blk, 0, s, p, b, g);
    launch_gbin_groups(g, b.n, s);
    GroupScratch g6 = g;
    g6.single = g.single6;
    g6.work = g.work6;
    if (p.snap) {
        if (v6) hipLaunchKernelGGL((k_deliver_runs<true, true>), grid, blk, 0, s, p, b, now, o, g6);
        else hipLaunchKernelGGL((k_deliver_runs<false, true>), grid, blk, 0, s, p, b, now, o, g);
    } else {
        if (v6) hipLaunchKernelGGL((k_deliver_runs<true, false>), grid, blk, 0, s, p, b, now, o, g6);
        else hipLaunchKernelGGL((k_deliver_runs<false, false>), grid, blk, 0, s, p, b, now, o, g);
    }
    hipLaunchKernelGGL(k_out_unpack, grid, blk, 0, s, o, g, b.n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// the stages after the front (service groups and LB positions, pairs, NAT links, the
// components and their CT / delivery positions) of one instance: EV the optional outputs,
// SN the saving of CT slots (egress admission with many CT maps).  Uses g.epoch and
// g.epoch + 1.
template <bool EV, bool SN>
void eg_stages(const DpParams &p, const BatchDev &b, const uint32_t *flow_hash, uint32_t now, const OutDev &o,
               GroupScratch g, hipStream_t s)
{
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    // the service groups (source, VIP) by binning, then one LB launch per member position
    {
        GroupScratch gl = g;
        gl.q4 = Q_LB4;
        gl.q6 = Q_LB6;
        gl.flat = 1;
        launch_gbin_groups(gl, b.n, s);
        GroupScratch gl6 = gl;
        gl6.work = g.work6;
        for (uint32_t k = 0; k < NPOS; ++k) {
            const dim3 gk(grid_for(b.n / (k + 1)));
            hipLaunchKernelGGL((k_lb_stage<false, EV, SN>), gk, blk, 0, s, p, b, flow_hash, now, o, gl, k);
            if (b.stride >= 128)
                hipLaunchKernelGGL((k_lb_stage<true, EV, SN>), gk, blk, 0, s, p, b, flow_hash, now, o, gl6, k);
        }
    }
    g.epoch += 1;
    if (b.stride >= 128) hipLaunchKernelGGL(k_egress_pairs<32>, grid, blk, 0, s, p, b, g);
    else hipLaunchKernelGGL(k_egress_pairs<16>, grid, blk, 0, s, p, b, g);
    hipLaunchKernelGGL(k_egress_nat, grid, blk, 0, s, p, b, g);
    hipLaunchKernelGGL(k_group_link, grid, blk, 0, s, b, g);
    g.q4 = Q_CT4;
    g.q6 = Q_CT6;
    g.flat = 1;
    launch_gbin_groups(g, b.n, s);
    // one launch per member position (the kernel boundary orders a group's members); a
    // list's length is at most n / (pos + 1)
    // and each followed by the local deliveries it handed over; the last (continuation)
    // list delivers inline
    for (uint32_t k = 0; k < NPOS; ++k) {
        const dim3 gk(grid_for(b.n / (k + 1)));
        GroupScratch gp = g, g6 = g;
        gp.pos = g6.pos = k;
        g6.work = g.work6;
        const bool last = k + 1 == NPOS;
        for (int v6 = 0; v6 < (b.stride >= 128 ? 2 : 1); ++v6) {
            const GroupScratch &gv = v6 ? g6 : gp;
            if (last) {
                if (v6) hipLaunchKernelGGL((k_egress_cont<true, EV, SN>), gk, blk, 0, s, p, b, now, o, gv, k);
                else hipLaunchKernelGGL((k_egress_cont<false, EV, SN>), gk, blk, 0, s, p, b, now, o, gv, k);
                continue;
            }
            if (v6) {
                hipLaunchKernelGGL((k_egress_ct<true, EV, false, SN>), gk, blk, 0, s, p, b, now, o, gv, k);
                hipLaunchKernelGGL((k_egress_deliver<true, EV, SN>), gk, blk, 0, s, p, b, now, o, gv);
            } else {
                hipLaunchKernelGGL((k_egress_ct<false, EV, false, SN>), gk, blk, 0, s, p, b, now, o, gv, k);
                hipLaunchKernelGGL((k_egress_deliver<false, EV, SN>), gk, blk, 0, s, p, b, now, o, gv);
            }
        }
    }
}

// ================================================================== launcher
// g.epoch .. g.epoch + 2 are used (service groups, conntrack groups, NAT writers).
int launch_lxc_egress(const DpParams &p, const BatchDev &b, const uint16_t *src_ep, uint32_t ep0,
                      const uint32_t *flow_hash, uint32_t now, const OutDev &o, GroupScratch g, hipStream_t s)
{
    g.lim = b.n;
    if (!b.n) return 0;
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    const bool ev = o.frames || p.notify || p.trace;              // the instance with the optional outputs
    if (b.stride >= 128) {
        if (ev) hipLaunchKernelGGL((k_egress_front<32, true>), grid, blk, 0, s, p, b, src_ep, ep0, o, g);
        else hipLaunchKernelGGL((k_egress_front<32, false>), grid, blk, 0, s, p, b, src_ep, ep0, o, g);
    } else {
        if (ev) hipLaunchKernelGGL((k_egress_front<16, true>), grid, blk, 0, s, p, b, src_ep, ep0, o, g);
        else hipLaunchKernelGGL((k_egress_front<16, false>), grid, blk, 0, s, p, b, src_ep, ep0, o, g);
    }
    if (ev) {
        if (p.snap) eg_stages<true, true>(p, b, flow_hash, now, o, g, s);
        else eg_stages<true, false>(p, b, flow_hash, now, o, g, s);
    } else {
        if (p.snap) eg_stages<false, true>(p, b, flow_hash, now, o, g, s);
        else eg_stages<false, false>(p, b, flow_hash, now, o, g, s);
    }
    g.epoch += 2;                                                 // (as eg_stages left its copy)
    g.q4 = Q_CT4;
    g.q6 = Q_CT6;
    g.flat = 1;
    hipLaunchKernelGGL(k_nat_group, grid, blk, 0, s, b, g);
    hipLaunchKernelGGL(k_nat_apply, grid, blk, 0, s, p, b, now, g);
    hipLaunchKernelGGL(k_out_unpack, grid, blk, 0, s, o, g, b.n);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cv
