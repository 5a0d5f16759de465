// cv_kernels.hip — gfx950 kernels of the batch verdict engine, ingress side.
//
// One lane = one packet.  Each kernel restates a path of the reference's BPF
// programs (Taeung/cilium v1.1.90) over a batch of frame records in HBM:
//   k_xdp_prefilter    bpf/bpf_xdp.c:88-184                      (config 1)
//   k_policy_ingress   bpf/bpf_netdev.c:128-153,357-398 +
//                      bpf/lib/policy.h:46-163                   (config 2)
//   k_netdev_front     bpf/bpf_netdev.c:357-524, bpf/lib/l3.h:103-132
//   k_ct_stage         bpf/bpf_lxc.c:865-1038, bpf/lib/conntrack.h (config 3)
// The egress path (config 5) is in cv_egress.hip; the shared device functions
// (map probes, policy, conntrack, metrics, grouping) in cv_dev.hpp.  No MFMA: this
// is integer gather work, HBM/L2 bound.
#include <type_traits>

#include "cv_dev.hpp"

namespace cv {

// the status of the launches just made: 0, or -EIO with the HIP error on stderr
static int launch_status(const char *where)
{
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    fprintf(stderr, "[cv] %s: %s\n", where, hipGetErrorString(e));
    return -5;
}

// ================================================================== config 1
// A wave's record load and probes: wave-cooperative 1-KiB record loads through LDS
// when the wave's 64 records are all in the batch (64-B stride), quad probes
// (cv_hash.hpp) for the tables; the loops are wave-uniform so every lane reaches
// every probe (lanes past the end with live = false).
__device__ __forceinline__ void rec_load_wave(Rec &r, const DpParams &p, const BatchDev &b, uint32_t i0, uint32_t i,
                                              bool live, uint4 *st)
{
    if (b.stride == 64 && i0 + 64 <= b.n) rec_load_wave64(r, b, i0, 4, st);
    else if (!live) { r.len = 0; for (int j = 0; j < 16; ++j) r.w[j] = 0; }
    else rec_load(r, b, i, 4);
}

// The config-2 verdict words leave as streaming (nontemporal) stores: the output
// lines are never read back by the launch, so they do not take L2 / Infinity Cache
// room from the table lines (config 2: 0.886 -> 0.870 ms, profiles/r01y/ab_nt*).
template <class T>
__device__ __forceinline__ void st_out(T *q, T v)
{
    __builtin_nontemporal_store(v, q);
}

__global__ void __launch_bounds__(BLOCK) k_xdp_prefilter(DpParams p, BatchDev b, OutDev o)
{
    __shared__ uint4 stage[BLOCK / 64][256];
    uint4 *st = stage[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < b.n; i0 += gridDim.x * BLOCK) {
        const uint32_t i = i0 + lane;
        const bool live = i < b.n;
        Rec r;
        rec_load_wave(r, p, b, i0, i, live, st);
        Acct a{0, 0};
        a.ctu = ct_unit(p);
        const uint8_t v = xdp_verdict_q(p, r, a, live, st);
        if (!live) continue;
        if (o.xdp) o.xdp[i] = v;                                 // (streaming byte stores: 1 % slower)
        if (o.reason) o.reason[i] = 0;
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
    const L4Hdr h = l4_read<34>(r, off);
    switch (proto) {
    case 1:                                                      // ICMP
        if (h.c1) return chk_err(h.c1, DROP_CT_INVALID_HDR);
        dport_raw = h.type == 8 ? 8u : 0u;                        // ECHO: sport = type, then reversed
        return 0;
    case 6:                                                      // TCP: flags then ports
        if (h.c14) return chk_err(h.c14, DROP_CT_INVALID_HDR);
        if (h.c4) return chk_err(h.c4, DROP_CT_INVALID_HDR);
        dport_raw = h.p2;
        return 0;
    case 17:                                                     // UDP
        if (h.c4) return chk_err(h.c4, DROP_CT_INVALID_HDR);
        dport_raw = h.p2;
        return 0;
    default:
        return DROP_CT_UNKNOWN_PROTO;
    }
}

// PPT packets per lane: lane t of workgroup w takes packets w*PPT*BLOCK + k*BLOCK + t
// (coalesced per k); its policy counter atomics wait in registers until its last
// lookup is done (2, 3, 5, 6 and 8 packets per lane measured slower).
constexpr int PPT = 4;

// The table probes are quad_find (cv_hash.hpp), so every lane of the wave reaches
// each probe; lanes without a lookup (past the batch end, non-IPv4, short or invalid
// headers) take part with want = false.  (Holding the results in registers until
// after the last probe, so the probes' vmcnt waits skip the output stores, measured
// 3 % slower.)
__global__ void __launch_bounds__(BLOCK) k_policy_ingress(DpParams p, int ep, BatchDev b, OutDev o)
{
    __shared__ unsigned long long drops[256 * 2];                 // ingress drops {count, bytes} by reason
    __shared__ uint4 stage[BLOCK / 64][256];
    for (int j = threadIdx.x; j < 256 * 2; j += BLOCK) drops[j] = 0;
    __syncthreads();
    const HashTable pol = G(p.eps)[ep].policy;
    uint4 *st = stage[threadIdx.x >> 6];
    Hit hits[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        hits[k] = Hit{nullptr, 0};
        const uint32_t i = blockIdx.x * (PPT * BLOCK) + k * BLOCK + threadIdx.x;
        const uint32_t i0 = i - (threadIdx.x & 63);
        if (i0 >= b.n) continue;                                  // the whole wave is past the end
        const bool live = i < b.n;
        Rec r;
        if (b.stride == 64 && i0 + 64 <= b.n) rec_load_wave64(r, b, i0, 3, st);
        else if (!live) { r.len = 0; for (int j = 0; j < 16; ++j) r.w[j] = 0; }
        else rec_load(r, b, i, 3);
        Acct a{0, 0};
        a.ctu = ct_unit(p);
        bool skip_proxy = false;
        uint32_t identity = 0;
        if (live && (p.flags & F_FROM_HOST)) identity = identity_from_mark(b.mark ? b.mark[i] : 0u, skip_proxy);
        const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
        const bool v4 = live && eth == 0x0008u && r.len >= 34;
        const bool want_ipc = v4 && identity < HEALTH_ID;         // bpf_netdev.c:375-398
        const uint32_t lab = ipcache4_q(p, rec_raw32c<26>(r), want_ipc, a, st);
        if (want_ipc && lab && lab != CLUSTER_ID && lab != HOST_ID) identity = lab;
        int32_t ret = eth != 0x0008u ? DROP_UNKNOWN_L3 : r.len < 34 ? DROP_INVALID : 0;
        uint32_t dport = 0, proto = 0;
        if (v4) ret = l4_key_new_flow(r, dport, proto);
        const bool want_pol = v4 && ret == 0;
        const int v = policy_ingress_q(pol, p.flags, r.len, identity, dport, proto, a, &hits[k], want_pol, st);
        uint16_t proxy = 0;
        if (v4 && ret == 0) {
            if (v < 0) ret = DROP_POLICY;
            else if (skip_proxy && v > 0) ret = 0;
            else { ret = v; proxy = v > 0 ? (uint16_t)v : 0; }
        }
        if (!live) continue;
        const bool dropped = ret < 0 && ret != E_TRUNC;
        if (dropped) {                                            // send_drop_notify -> cilium_metrics
            const uint32_t rr = (uint8_t)(-ret);
            atomicAdd(&drops[2 * rr], 1ull);
            atomicAdd(&drops[2 * rr + 1], (unsigned long long)r.len);
        }
        if (o.ret) st_out(o.ret + i, ret);
        if (o.identity) st_out(o.identity + i, identity);
        if (o.reason) o.reason[i] = dropped ? ret : 0;
        if (o.proxy) o.proxy[i] = proxy;
        if (o.ct) o.ct[i] = CT_NONE;
        store_out(o, i, a);
    }
#pragma unroll
    for (int k = 0; k < PPT; ++k) hit_flush(hits[k]);
    __syncthreads();
    if (p.metrics)                                                // (no forwards are counted on this path)
        for (int j = threadIdx.x; j < 256; j += BLOCK)
            if (drops[2 * j]) {
                atomicAdd(&p.metrics[(j * 4 + METRIC_INGRESS) * 2], drops[2 * j]);
                atomicAdd(&p.metrics[(j * 4 + METRIC_INGRESS) * 2 + 1], drops[2 * j + 1]);
            }
}

// ================================================================== config 3
// handle_ipv6 of bpf_netdev (bpf_netdev.c:172-276; HANDLE_NS, FROM_HOST, no
// ENCAP_IFINDEX, reverse_proxy6 with an empty cilium_proxy6 map) up to the tail call
// into the endpoint's policy program.  Per-lane probes (IPv6 is the rare family on
// this path).  Returns the verdict code of a packet that stops here; *stage: the
// packet goes on to ipv6_policy; *rw: rewrite_dmac_to_host ran; *ldabs: icmp6_load_type
// read past the packet, which ends the program with 0 (TC_ACT_OK, no notification).
template <int NW>
__device__ __forceinline__ int netdev_ipv6(const DpParams &p, const RecT<NW> &r, uint32_t &identity, Acct &a,
                                           uint32_t &flowlabel, bool &stage, int64_t &slot, uint32_t &iv, bool &rw,
                                           bool &ldabs)
{
    stage = rw = ldabs = false;
    slot = -1;
    iv = 0;
    if (r.len < 54) return DROP_INVALID;                          // revalidate_data
    uint32_t nh = rec_u8c<20>(r);
    const int hl = ipv6_hdrlen(r, nh);
    if (hl < 0) return hl;
    const int l4 = 14 + hl;
    const uint32_t sa[4] = {rec_raw32c<22>(r), rec_raw32c<26>(r), rec_raw32c<30>(r), rec_raw32c<34>(r)};
    const uint32_t da[4] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r)};
    if (nh == 58) {                                               // icmp6_handle (icmp6.h:390-412)
        const int c = rec_chk(r, 54, 1);                          // icmp6_load_type: load_byte(ETH_HLEN + 40)
        if (c == E_TRUNC) return E_TRUNC;
        if (c) { ldabs = true; return TC_ACT_OK; }
        const uint32_t type = rec_u8c<54>(r);
        if (type == 135 || (type == 128 && eq4(da, p.router6))) return E_PUNT;   // NS / echo to the router
    }
    if (identity < HEALTH_ID) {                                   // identity_is_reserved (policy.h:46-49)
        const uint32_t lab = ipcache6(p, sa, a);
        if (lab && lab != CLUSTER_ID) identity = lab;
    }
    flowlabel = WORLD_ID;                                         // derive_sec_ctx (:50-64)
    if (sa[0] == p.router6[0] && sa[1] == p.router6[1]) flowlabel = bswap32(rec_raw32c<14>(r)) & 0x000FFFFFu;
    if (p.flags & F_FROM_HOST) {
        flowlabel = identity;
        const uint32_t nh0 = rec_u8c<20>(r);                      // reverse_proxy6 gets ip6->nexthdr
        if (nh0 == 6 || nh0 == 17) {
            const int c = rec_chk(r, l4, 4);
            if (c) return chk_err(c, DROP_CT_INVALID_HDR);
        }
        rw = true;                                                // rewrite_dmac_to_host
    }
    if (!p.lxc6.buckets) return TC_ACT_OK;
    a.nl++;                                                       // lookup_ip6_endpoint
    slot = dev_find<LxcV6Spec>(p.lxc6, da, &iv);
    if (slot < 0 || (iv & (1u << 16))) return TC_ACT_OK;          // not local / ENDPOINT_F_HOST
    if (rec_u8c<21>(r) <= 1) return E_PUNT;                       // ipv6_l3: icmp6_send_time_exceeded
    const uint32_t e = p.ep_of_lxc ? p.ep_of_lxc[iv & 0xFFFFu] : 0u;
    if (!e) return DROP_MISSED_TAIL_CALL;
    stage = true;                                                 // ipv6_local_delivery -> handle_policy
    return TC_ACT_OK;
}

constexpr uint64_t SALT_NETDEV6 = 0x4E45543600000000ULL;

// Occupancy of the netdev front and conntrack stage (waves per SIMD the compiler must
// allow; 0: its own choice, 4 at 107-110 VGPRs)
#ifndef CV_NS_WAVES
#define CV_NS_WAVES 0
#endif
#if CV_NS_WAVES
#define CV_NS_OCC __attribute__((amdgpu_waves_per_eu(CV_NS_WAVES, 8)))
#else
#define CV_NS_OCC
#endif

// stage 1: XDP prefilter + from_netdev -> handle_ipv4 / handle_ipv6 up to the tail call
// into the endpoint's policy program; packets reaching it join their address-pair
// group (IPv4 in Q_NETDEV, IPv6 in Q_NETDEV6).
template <bool EV>
__global__ void __launch_bounds__(BLOCK) CV_NS_OCC k_netdev_front(DpParams p, BatchDev b, OutDev o, GroupScratch g,
                                                        int with_prefilter)
{
    __shared__ LdsMetrics lm;
    __shared__ uint4 stage[BLOCK / 64][256];
    uint4 *st = stage[threadIdx.x >> 6];
    using M = MetT<EV>;
    M m;
    met_init(m, lm);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < b.n; i0 += gridDim.x * BLOCK) {
        const uint32_t i = i0 + lane;
        const bool live = i < b.n;
        Rec r;
        rec_load_wave(r, p, b, i0, i, live, st);
        Acct a{0, 0};
        a.ctu = ct_unit(p);
        uint8_t xv = XDP_PASS;
        int32_t ret = TC_ACT_OK, reason = 0;
        uint32_t ident = 0;
        bool staged = false, v6stage = false, dmac_rw = false;
        int64_t lxc_slot = -1;
        uint32_t iv = 0;
        if (with_prefilter) xv = xdp_verdict_q(p, r, a, live, st, &lxc_slot, &iv);
        const bool pass = live && xv == XDP_PASS;
        bool skip_proxy = false;
        uint32_t identity = 0;
        uint32_t smeta = 0, slabel = 0;                           // the hand-over to the policy program
        if (pass && (p.flags & F_FROM_HOST)) identity = identity_from_mark(b.mark ? b.mark[i] : 0u, skip_proxy);
        ident = identity;
        if (EV && pass && p.trace) {                              // from_netdev: send_trace_notify(FROM_*)
            const uint32_t mg = (b.mark ? b.mark[i] : 0u) & 0xF00u;
            const uint32_t obs = !(p.flags & F_FROM_HOST) ? TRACE_FROM_STACK
                                 : (mg == 0xA00u || mg == 0xB00u) ? TRACE_FROM_PROXY : TRACE_FROM_HOST;
            m.pkt = b.base + i;
            m.hash = b.hash ? b.hash[i] : 0u;
            notify_trace(p, m, obs, r.len, 0, identity, 0, 0, p.ingress_ifindex, 0, true);
        }
        const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
        const bool v4 = pass && eth == 0x0008u && r.len >= 34;   // handle_ipv4 (bpf_netdev.c:357-453)
        const uint32_t nexthdr = rec_u8c<23>(r);
        const int l4 = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
        uint32_t secctx = WORLD_ID;
        const bool want_ipc = v4 && identity < HEALTH_ID;
        const uint32_t lab = ipcache4_q(p, rec_raw32c<26>(r), want_ipc, a, st);
        if (want_ipc && lab && lab != CLUSTER_ID && lab != HOST_ID) identity = lab;
        int h = TC_ACT_OK;
        if (v4) {
            ident = identity;
            if (p.flags & F_FROM_HOST) {
                secctx = identity;
                if (nexthdr == 6 || nexthdr == 17) {              // reverse_proxy port load
                    const int c = rec_chk(r, l4, 4);
                    if (c) h = chk_err(c, DROP_CT_INVALID_HDR);
                }
                dmac_rw = h == TC_ACT_OK;                         // rewrite_dmac_to_host (:156-169)
            }
        }
        const bool want_lxc = v4 && h == TC_ACT_OK && p.lxc4.buckets;
        if (want_lxc) a.nl++;                                     // lookup_ip4_endpoint
        uint32_t daddr = rec_raw32c<30>(r);
        // with the prefilter, an IPv4 packet got here only after check_v4_endpoint
        // found its daddr in the same table: that probe's answer is reused (read-only
        // within the launch); without it, one quad probe (wave-uniform branch)
        if (!with_prefilter) lxc_slot = quad_find<LxcV4Spec>(p.lxc4, &daddr, want_lxc, st, &iv);
        const bool lxc_hit = lxc_slot >= 0;
        if (pass && eth == 0x0008u) {
            if (r.len < 34) {
                h = DROP_INVALID;
            } else if (want_lxc && lxc_hit) {
                if (iv & (1u << 16)) {
                    h = TC_ACT_OK;                                // ENDPOINT_F_HOST
                } else if (rec_u8c<22>(r) <= 1) {
                    h = DROP_INVALID;                             // ipv4_dec_ttl
                } else {
                    const uint32_t e = p.ep_of_lxc ? p.ep_of_lxc[iv & 0xFFFFu] : 0u;
                    if (!e) {
                        h = DROP_MISSED_TAIL_CALL;
                    } else {
                        staged = true;                            // -> handle_policy -> tail_ipv4_policy
                        slabel = secctx;
                        smeta = (e - 1) | (skip_proxy ? 1u << 16 : 0u) | ((iv >> 17) & 1u) << 17;
                        if (EV) g.ifx[i] = (uint32_t)lxc_slot;    // -> cb[CB_IFINDEX], MACs (stage 2)
                    }
                }
            }
        } else if (pass && eth == 0xDD86u) {                      // handle_ipv6 (bpf_netdev.c:172-276)
            uint32_t flowlabel = WORLD_ID;
            bool ldabs;
            h = netdev_ipv6(p, r, identity, a, flowlabel, v6stage, lxc_slot, iv, dmac_rw, ldabs);
            ident = identity;
            if (ldabs) { h = TC_ACT_OK; dmac_rw = false; }
            if (v6stage) {
                const uint32_t e = p.ep_of_lxc[iv & 0xFFFFu];
                slabel = flowlabel;
                smeta = (e - 1) | (skip_proxy ? 1u << 16 : 0u) | ((iv >> 17) & 1u) << 17;
                if (EV) g.ifx[i] = (uint32_t)lxc_slot;
            }
        }
        if ((pass && eth == 0x0008u) || (pass && eth == 0xDD86u)) {
            if (!staged && !v6stage) {
                if (h == E_TRUNC || h == E_PUNT) ret = h;
                else if (is_err(h)) {                             // tail_handle_ipv4 / from_netdev:
                    m.drop(h, r.len, METRIC_INGRESS);             // send_drop_notify_error
                    m.pkt = b.base + i;
                    m.hash = b.hash ? b.hash[i] : 0u;
                    notify_drop(p, m, h, r.len, 0, 0, 0, 0, 0);
                    reason = h;
                    ret = TC_ACT_SHOT;
                }
                else ret = h;
            }
        }
        // the group key (CT map, address pair) of a packet handed to the policy program:
        // bit 0 = its queue (0 IPv4, 1 IPv6), bit 1 set (never 0); k_gbin_group bins and
        // groups by it
        unsigned long long gkey = 0;
        if (staged) {
            const uint32_t ct_id = (p.uni4_on ? p.uni4.ct_v4 : G(p.ephot)[smeta & 0xFFFFu].ct_v4) & EPH_CT_ID;
            gkey = (pair_hash4(rec_raw32c<26>(r), daddr, (uint64_t)ct_id << 17) & ~3ull) | 2ull;
        } else if (v6stage) {
            const EpDev ep = G(p.eps)[smeta & 0xFFFFu];
            const uint32_t sa[4] = {rec_raw32c<22>(r), rec_raw32c<26>(r), rec_raw32c<30>(r), rec_raw32c<34>(r)};
            const uint32_t da[4] = {rec_raw32c<38>(r), rec_raw32c<42>(r), rec_raw32c<46>(r), rec_raw32c<50>(r)};
            gkey = (pair_hash6(sa, da, SALT_NETDEV6 ^ (uint64_t)(uintptr_t)ep.ct6.buckets) & ~3ull) | 3ull;
        }
        if (p.flags & F_TEST_COARSE_GROUPS) gkey &= 0xFF00000000000003ull;
        if (!live) continue;
        g.pkey[i] = gkey;
        g.hword[i] = 0;
        g.gslot[i] = NONE;
        const bool fwd_here = !staged && !v6stage && ret == TC_ACT_OK;
        if (M::EV && o.frames) {
            uint8_t *fo = o.frames + (size_t)i * b.stride;
            frame_copy(b.frames + (size_t)i * b.stride, fo, b.stride);
            if (fwd_here && dmac_rw) {                            // the forwarded frame's new dmac
                *reinterpret_cast<uint32_t *>(fo) = p.net_mac[0];
                *reinterpret_cast<uint16_t *>(fo + 4) = (uint16_t)p.net_mac[1];
            }
        }
        if (!staged && !v6stage) {
            if (o.ret) o.ret[i] = ret;
            if (o.reason) o.reason[i] = reason;
            if (o.ct) o.ct[i] = CT_NONE;
            if (o.proxy) o.proxy[i] = 0;
            store_out(o, i, a);
        } else {                                                  // the stage record (stage 2 adds its accounting)
            uint32_t w4 = 0, chk = 0;
            if (staged) g.srec[2 * i] = skb4_pack(skb4_from(r), w4, chk);
            g.srec[2 * i + 1] = make_uint4(w4, chk | (a.nl & 0xFFu) << 16 | (a.nu & 0xFFu) << 24, smeta, slabel);
        }
        if (o.xdp) o.xdp[i] = xv;
        if (o.identity) o.identity[i] = ident;
    }
    met_flush(m, p.metrics);
}

template <class M>
__device__ __forceinline__ void stage2_one(const DpParams &p, const BatchDev &b, const OutDev &o,
                                           const GroupScratch &g, uint32_t i, uint32_t now, M &m, bool single)
{
    const uint4 s0 = g.srec[2 * i], s1 = g.srec[2 * i + 1];
    const uint32_t meta = s1.z;
    const EpDev ep = ep_netdev4<M::EV>(p, meta & 0xFFFFu);
    Acct a{(s1.y >> 16) & 0xFFu, s1.y >> 24, m.pc};
    a.ctu = ct_unit(p);
    uint8_t ct = CT_NONE;
    uint16_t proxy = 0;
    int32_t reason = 0;
    Skb4 s = skb4_unpack(s0, s1.x, s1.y & 0x3FFu, b.stride);
    int64_t lslot = -1;                                          // the destination's cilium_lxc slot
    if constexpr (M::EV) {
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        lslot = (int32_t)g.ifx[i];
    }
    RevNatOut rn{false, false, 0, 0};
    if (p.budget) a.budget = p.budget[i];                        // (admission windows)
    // the only packet of its group defers its create to k_ct_commit (not with event
    // records, whose TRACE_TO_LXC would have to be withdrawn if the create failed, nor
    // with a budget short of the tuple and its twin)
    bool defer = single && !p.ct_guard && !M::EV && a.budget >= 2;
    const int ret = handle_policy4<M, false>(p, ep, s, s1.w, (meta >> 16) & 1u,
                                   ifindex_of(m, p.lxc4, lslot, ((meta >> 17) & 1u) << 17), now, ct, proxy, reason,
                                   a, m, &rn, &defer);
    if (defer) g.gslot[i] = proxy ? COMMIT4 - COMMIT_PROXY : COMMIT4;
    if (M::EV && o.frames && (ret == TC_ACT_OK || ret == TC_ACT_REDIRECT) && !proxy) {
        // the forwarded frame: ipv4_local_delivery's ipv4_l3 (bpf_netdev handle_ipv4), then
        // the policy program's reverse NAT
        const uint8_t *in = b.frames + (size_t)i * b.stride;
        Rec r;
        rec_load(r, b, i, 3);
        Frame4 f;
        frame4_init(f, r, in);
        uint32_t mac[2], nmac[2];
        lxc_macs(p.lxc4, lslot, mac, nmac);
        frame4_l3(f, nmac, mac);
        if (rn.valid) frame4_revnat(f, rn.na, rn.np, false, f.saddr);
        frame4_emit(f, in, o.frames + (size_t)i * b.stride, b.stride, r.len);
    }
    if (o.ret) o.ret[i] = ret;
    if (o.reason) o.reason[i] = reason;
    if (o.ct) o.ct[i] = ct;
    if (o.proxy) o.proxy[i] = proxy;
    store_out(o, i, a);
}

// ------------------------------------------------------------------ hot runs
// A group of many packets (an elephant flow: one address pair carrying thousands of
// the batch's packets) walked by one lane costs a chain of dependent memory round trips
// per member.  Runs of size class >= HOT_CLASS (more than 32 members) go to k_ct_hot, a
// workgroup of HOTB threads per run, HOTB members at a time:
//  1. every thread looks its member up against the table as the chunk starts (read
//     only: ct_lookup_pre, policy_ingress_denies) and tells whether its ipv4_policy
//     would change which keys exist -- a create (CT_NEW, allowed) or a delete
//     (CT_ESTABLISHED, denied);
//  2. the members before the first such one (c) change no key, so each sees exactly
//     what the sequential run shows it: they finish in parallel (verdicts, policy
//     counters, metrics), their hits' entry updates deferred;
//  3. the deferred updates of one entry are folded in parallel (hot_fold): what an update
//     does next depends on the entry only through three bits (RX / TX closing, seen
//     non-SYN), so every member's update is an 8-state transition table, a block scan of
//     their compositions gives each member the bits it meets, and the rest of the entry
//     is a reduction -- the lifetime of the last update that set one, the OR of the
//     flags seen per direction, the report stamps, the counter sums;
//  4. member c runs whole (its create or delete), then the next chunk starts after it.
// An elephant flow's established packets all take step 2 and 3: a chunk of HOTB members
// costs one round of lookups and a scan.  Only the plain instance (no event records,
// whose trace decisions need the per-packet entry state) and launches without admission
// budgets or guards use it; the others keep one lane per run.
#ifndef CV_HOT_CLASS
#define CV_HOT_CLASS 14
#endif
constexpr int HOT_CLASS = CV_HOT_CLASS;                           // size_class: runs of more than 128 members
                                                                  // (12 / 13: 32 / 64 measured 13 % / 2 % slower on Zipf 1.1)
constexpr uint32_t HOTB = 1024;                                   // threads (members) per chunk
constexpr uint32_t HOT_ENTRIES = 16;                              // entries one chunk may fold

__device__ __forceinline__ uint32_t hot_runs(const GroupScratch &g, int q)
{
    uint32_t n = 0;
#pragma unroll
    for (int c = HOT_CLASS; c < NCLASS; ++c) n += g.cursor[qcls(q, c)];
    return n;
}

// The hit update ct_hit_apply (conntrack.h:213-258) as a function of the three bits it
// reads, x = RX_CLOSING | TX_CLOSING << 1 | SEEN_NON_SYN << 2: the bits it leaves, whether
// it ran __ct_update_timeout at all (every run uses the member's direction and flags) and
// the lifetime of its last run.
struct HitFx {
    uint32_t x, any, life;
};

__device__ __forceinline__ HitFx hit_fx(uint32_t x, uint32_t action, uint32_t dir, uint32_t tcp, uint32_t seen)
{
    HitFx f{x, 0u, 0u};
    auto alive = [&]() { return (f.x & 3u) != 3u; };
    auto timeout = [&]() {                                        // ct_update_timeout (conntrack.h:169-186)
        if (tcp && !(seen & TCPF_SYN)) f.x |= 4u;
        f.life = tcp ? ((f.x & 4u) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT) : CT_LIFETIME_NONTCP;
        f.any = 1u;
    };
    if (alive()) timeout();
    if (action == ACTION_CREATE) {
        if (f.x & 3u) { f.x &= ~3u; timeout(); }
    } else if (action == ACTION_CLOSE) {
        f.x |= dir == CT_INGRESS ? 1u : 2u;
        if (!alive()) { f.life = CT_CLOSE_TIMEOUT; f.any = 1u; }  // __ct_update_timeout(CT_CLOSE_TIMEOUT)
    }
    return f;
}

constexpr uint32_t FX_IDENT = 0u | 1u << 3 | 2u << 6 | 3u << 9 | 4u << 12 | 5u << 15 | 6u << 18 | 7u << 21;
__device__ __forceinline__ uint32_t fx_at(uint32_t T, uint32_t x) { return (T >> (3 * x)) & 7u; }
__device__ __forceinline__ uint32_t fx_then(uint32_t A, uint32_t B)   // A, then B
{
    uint32_t r = 0;
#pragma unroll
    for (uint32_t x = 0; x < 8; ++x) r |= fx_at(B, fx_at(A, x)) << (3 * x);
    return r;
}
__device__ __forceinline__ uint32_t bits_x(uint32_t b)
{
    return (b & CTB_RX_CLOSING ? 1u : 0u) | (b & CTB_TX_CLOSING ? 2u : 0u) | (b & CTB_SEEN_NON_SYN ? 4u : 0u);
}

struct HotLds {
    uint32_t c, lead, wscan[HOTB / 64], fxtot, fxlast, seen[2], any[2];
    unsigned long long slot;
    uint32_t pk[2], by[2];                                        // (a chunk's sums fit 32 bits)
    uint32_t e[CT_HOTW];                                          // the folded entry's hot run (h0..h9)
};

// the block's exclusive scan of transition tables in thread order (its total in *tot)
__device__ __forceinline__ uint32_t fx_scan(uint32_t T, HotLds &L, uint32_t *tot)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t incl = T;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, d, 64);
        if (lane >= (uint32_t)d) incl = fx_then(t, incl);
    }
    if (lane == 63) L.wscan[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = FX_IDENT;
        for (uint32_t w = 0; w < nw; ++w) { const uint32_t t = L.wscan[w]; L.wscan[w] = acc; acc = fx_then(acc, t); }
        L.fxtot = acc;
    }
    __syncthreads();
    uint32_t ex = (uint32_t)__shfl_up((int)incl, 1, 64);
    if (lane == 0) ex = FX_IDENT;
    const uint32_t r = fx_then(L.wscan[wv], ex);
    *tot = L.fxtot;
    __syncthreads();
    return r;
}

// the folded hot run written back: the three state bits the updates leave (x1), the
// lifetime of the last update that set one (lc: 1 TCP, 2 close, 0 otherwise; valid), the
// report stamps and flags seen per direction, the counter sums (carries to the side slot)
__device__ __forceinline__ void hot_store(const HashTable &ct, int64_t slot, uint32_t *h, uint32_t x1, bool lvalid,
                                          uint32_t lc, const uint32_t *seen, const uint32_t *any,
                                          const unsigned long long *pk, const unsigned long long *by, uint32_t now,
                                          uint32_t flags)
{
    uint32_t b = h[1] & ~(uint32_t)(CTB_RX_CLOSING | CTB_TX_CLOSING | CTB_SEEN_NON_SYN);
    b |= (x1 & 1u ? CTB_RX_CLOSING : 0u) | (x1 & 2u ? CTB_TX_CLOSING : 0u) | (x1 & 4u ? CTB_SEEN_NON_SYN : 0u);
    h[1] = b;
    if (lvalid) h[0] = now + (lc == 1u ? CT_LIFETIME_TCP : lc == 2u ? CT_CLOSE_TIMEOUT : CT_LIFETIME_NONTCP);
    for (int d = 0; d < 2; ++d) {                                 // __ct_update_timeout's reports (0 tx, 1 rx)
        if (!any[d]) continue;
        const int fsh = d ? 24 : 16, li = d ? 5 : 4;               // rx_flags_seen / tx_flags_seen; last_rx / tx_report
        const uint32_t acc = (h[2] >> fsh) & 0xFFu, nacc = acc | seen[d];
        if (h[li] + CT_REPORT_INTERVAL < now || nacc != acc) {
            h[li] = now;
            h[2] = (h[2] & ~(0xFFu << fsh)) | (nacc << fsh);
        }
    }
    CtE e;
    e.w[8] = h[0]; e.w[9] = h[1]; e.w[10] = h[2]; e.w[11] = h[3]; e.w[12] = h[4]; e.w[13] = h[5];
    e.w[0] = h[6]; e.w[2] = h[7]; e.w[4] = h[8]; e.w[6] = h[9];
    if (flags & F_CT_ACCOUNTING) {                                // ct_count: low words in place, carries to the side slot
        for (int d = 0; d < 2; ++d) {
            const int k0 = d ? 0 : 4;                              // rx_packets / rx_bytes @0 / 2, tx @4 / 6
            const unsigned long long sp = (unsigned long long)e.w[k0] + pk[d];
            const unsigned long long sb = (unsigned long long)e.w[k0 + 2] + by[d];
            e.w[k0] = (uint32_t)sp;
            e.w[k0 + 2] = (uint32_t)sb;
            CV_G uint32_t *cold = ct_cold<Ct4Spec>(ct, slot);
            if (sp >> 32) cold[k0 >> 1] += (uint32_t)(sp >> 32);
            if (sb >> 32) cold[(k0 + 2) >> 1] += (uint32_t)(sb >> 32);
        }
    }
    ct_store_hot<Ct4Spec>(ct, slot, e);
}

// step 3 for the entry at L.slot: the deferred hits of the participating threads (in
// thread = member order) applied as the sequential run applies them one by one
template <class S>
__device__ __forceinline__ void hot_load(const HashTable &ct, HotLds &L, int64_t slot)
{
    CtE e;
    ct_load_hot<S>(ct, slot, e);
    L.e[0] = e.w[8]; L.e[1] = e.w[9]; L.e[2] = e.w[10]; L.e[3] = e.w[11]; L.e[4] = e.w[12]; L.e[5] = e.w[13];
    L.e[6] = e.w[0]; L.e[7] = e.w[2]; L.e[8] = e.w[4]; L.e[9] = e.w[6];
}

// (loaded: L.e already holds the entry's hot run -- the chunk's first entry, loaded by its
// first member's thread while the others finish their packets)
template <class S>
__device__ __forceinline__ void hot_fold(const HashTable &ct, HotLds &L, bool part, const HitRec &hr, uint32_t now,
                                         uint32_t flags, bool loaded)
{
    const int64_t slot = (int64_t)L.slot;
    if (threadIdx.x == 0) {
        if (!loaded) hot_load<S>(ct, L, slot);
        L.fxlast = 0; L.seen[0] = L.seen[1] = 0; L.any[0] = L.any[1] = 0;
        L.pk[0] = L.pk[1] = L.by[0] = L.by[1] = 0;
    }
    __syncthreads();
    uint32_t T = FX_IDENT;
    if (part) {
        T = 0;
#pragma unroll
        for (uint32_t x = 0; x < 8; ++x) T |= hit_fx(x, hr.action, hr.dir, hr.tcp, hr.seen).x << (3 * x);
    }
    uint32_t tot;
    const uint32_t pre = fx_scan(T, L, &tot);                    // (ends with a barrier)
    const uint32_t x0 = bits_x(L.e[1] & 0xFFFFu);
    const bool rx = hr.dir == CT_INGRESS;
    // the reductions per wave first (shuffles), then one LDS atomic per wave and word: the
    // members of a hot run all update one entry, so per-lane atomics would serialise on
    // the same LDS words
    uint32_t last = 0, sn[2] = {0u, 0u}, an[2] = {0u, 0u}, pk[2] = {0u, 0u}, by[2] = {0u, 0u};
    if (part) {
        const HitFx f = hit_fx(fx_at(pre, x0), hr.action, hr.dir, hr.tcp, hr.seen);
        const int d = rx ? 1 : 0;
        if (f.any) {
            last = (threadIdx.x + 1) << 8 | (f.life == CT_LIFETIME_TCP ? 1u : f.life == CT_CLOSE_TIMEOUT ? 2u : 0u);
            sn[d] = hr.seen & 0xFFu;
            an[d] = 1u;
        }
        if (flags & F_CT_ACCOUNTING) { pk[d] = 1u; by[d] = hr.len; }
    }
#pragma unroll
    for (int k = 32; k; k >>= 1) {
        last = max(last, (uint32_t)__shfl_xor((int)last, k, 64));
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            sn[d] |= (uint32_t)__shfl_xor((int)sn[d], k, 64);
            an[d] |= (uint32_t)__shfl_xor((int)an[d], k, 64);
            pk[d] += (uint32_t)__shfl_xor((int)pk[d], k, 64);
            by[d] += (uint32_t)__shfl_xor((int)by[d], k, 64);
        }
    }
    if ((threadIdx.x & 63) == 0) {
        if (last) atomicMax(&L.fxlast, last);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            if (an[d]) { atomicOr(&L.seen[d], sn[d]); atomicOr(&L.any[d], 1u); }
            if (pk[d]) { atomicAdd(&L.pk[d], pk[d]); atomicAdd(&L.by[d], by[d]); }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long pk[2] = {L.pk[0], L.pk[1]}, by[2] = {L.by[0], L.by[1]};
        hot_store(ct, slot, L.e, fx_at(tot, x0), L.fxlast != 0, L.fxlast & 0xFFu, L.seen, L.any, pk, by, now, flags);
    }
    __syncthreads();
}

// ipv4_policy (bpf_lxc.c:865-979) of a member that creates and deletes nothing: its
// lookup (ct_lookup_pre) hit -- the entry update deferred to the fold -- or missed with
// a denying policy
template <class M>
__device__ __forceinline__ int hot_finish(const DpParams &p, const EpDev &ep, Skb4 &s, Tuple4 &t, int ret,
                                          const CtState &st, uint32_t src_label, bool skip_proxy, uint32_t ifindex,
                                          uint8_t &ct_out, uint16_t &proxy, int32_t &reason, Acct &a, M &m)
{
    if (ret >= 0) {
        ct_out = (uint8_t)ret;
        if (ret == CT_REPLY && st.rev_nat && !st.loopback) {     // lb4_rev_nat(REV_NAT_F_TUPLE_SADDR)
            uint32_t na, np;
            if (revnat4(p, st.rev_nat, na, np, a)) {
                const int r2 = rev_map_port(s.h, t.nexthdr, np);
                const int r3 = r2 ? 0 : l4_csum_err(s, t.nexthdr);
                if (r2 || r3) ret = r2 ? r2 : r3;
                else t.saddr = na;
            }
        }
    }
    if (ret >= 0) {
        int verdict = policy_ingress<false>(ep.policy, p.flags, s.len, src_label, t.dport, t.nexthdr, a);
        if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
            ret = DROP_POLICY;                                    // (a miss: an established one would delete)
        } else {
            if (skip_proxy) verdict = 0;
            if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
                proxy = (uint16_t)verdict;                        // ipv4_redirect_to_host_port
                return TC_ACT_REDIRECT;
            }
            m.fwd(s.len, METRIC_INGRESS);                         // send_trace_notify(TRACE_TO_LXC)
            return ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
        }
    }
    if (ret == E_TRUNC) return ret;
    m.drop(ret, s.len, METRIC_INGRESS);                           // tail_ipv4_policy: send_drop_notify
    reason = ret;
    return TC_ACT_SHOT;
}

// One member of a hot run: its stage record and its lookups against the table as the
// chunk starts (read only: ct_lookup_pre, policy_ingress_denies), and whether its
// ipv4_policy would change which keys exist -- a create (CT_NEW, allowed) or a delete
// (CT_ESTABLISHED, denied) -- or it is on another CT map than the run's first member
// (two groups merged by a key collision: endpoints with their own maps): such a member
// runs whole.
struct HotMember {
    uint32_t x;
    bool live, simple, change;
    uint4 s1;
    EpDev ep;
    Skb4 s;
    Tuple4 t;
    CtState st;
    HitRec hr;
    int ret;
};

__device__ __forceinline__ void hot_lookup(const DpParams &p, const BatchDev &b, const GroupScratch &g,
                                           const HashTable &ct, uint32_t off, uint32_t cnt, uint32_t k, HotMember &h,
                                           Acct &a)
{
    h.x = k < cnt ? g.order[off + 1 + k] : 0u;
    h.live = k < cnt && pkt_ok(g, h.x);
    if (!h.live) h.x = 0u;
    uint4 s0{};
    h.s1 = uint4{};
    if (h.live) { s0 = g.srec[2 * h.x]; h.s1 = g.srec[2 * h.x + 1]; }
    const uint32_t meta = h.s1.z;
    h.ep = ep_netdev4<false>(p, meta & 0xFFFFu);
    h.s = skb4_unpack(s0, h.s1.x, h.s1.y & 0x3FFu, b.stride);
    h.simple = h.live && !(p.flags & F_DROP_ALL) && h.ep.ipv4 && h.s.len >= 34;
    a = Acct{(h.s1.y >> 16) & 0xFFu, h.s1.y >> 24, a.pc};
    h.t = Tuple4{};
    h.t.nexthdr = h.s.nexthdr; h.t.daddr = h.s.daddr; h.t.saddr = h.s.saddr;
    h.st = CtState{0, 0, 0, 0, 0, 0};
    h.hr = HitRec{-1, 0, 0, 0, 0, 0};
    int64_t slot = -1;
    h.ret = h.simple ? ct_lookup_pre(h.ep.ct4, h.t, h.s.h, CT_INGRESS, h.s.len, slot, &h.st, a, h.hr) : 0;
    const bool deny = h.simple && h.ret >= 0 &&
                      policy_ingress_denies(h.ep.policy, p.flags, h.s1.w, h.t.dport, h.t.nexthdr);
    const bool other_map = h.simple && h.ep.ct4.buckets != ct.buckets;
    h.change = h.simple && (other_map || (h.ret == CT_ESTABLISHED && deny) || (h.ret == CT_NEW && !deny));
}

// a member before the chunk's first change, whole: its lookup hit (the entry update
// deferred to the fold) or missed with a denying policy, or it drops before any
// conntrack work
template <class M>
__device__ __forceinline__ void hot_member_finish(const DpParams &p, const OutDev &o, HotMember &h, Acct &a, M &m,
                                                  uint32_t now)
{
    uint8_t ct = CT_NONE;
    uint16_t proxy = 0;
    int32_t reason = 0;
    const bool skip_proxy = (h.s1.z >> 16) & 1u;
    const uint32_t ifx = (h.s1.z >> 17) & 1u;                     // ifindex != 0 (the plain instance's view)
    int rv;
    if (h.simple) {
        rv = hot_finish(p, h.ep, h.s, h.t, h.ret, h.st, h.s1.w, skip_proxy, ifx, ct, proxy, reason, a, m);
    } else {
        a = Acct{(h.s1.y >> 16) & 0xFFu, h.s1.y >> 24, a.pc};
        rv = handle_policy4<M, false>(p, h.ep, h.s, h.s1.w, skip_proxy, ifx, now, ct, proxy, reason, a, m);
    }
    if (o.ret) o.ret[h.x] = rv;
    if (o.reason) o.reason[h.x] = reason;
    if (o.ct) o.ct[h.x] = ct;
    if (o.proxy) o.proxy[h.x] = proxy;
    store_out(o, h.x, a);
}


__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, uint32_t &total);

// ------------------------------------------------------------------ elephants in parallel
// A run of at least HPAR_MIN members (an elephant flow's address pair) is walked by
// k_ct_hot a chunk of HOTB members at a time, and its chunks are sequential.  But up to
// the run's first member that changes a key (or hits a second entry), every member sees
// the table as the launch found it, so the chunks before it need not wait for each other:
//  k_hpar_look  the elephants among the first HPAR_RUNS hot runs, their chunks numbered;
//               per chunk (a workgroup each, all at once): the lookups, the first change,
//               the first hit and its entry, the first hit on another entry;
//  k_hpar_fin   per chunk: the elephant's entry e (its first hit's) and its cut -- the
//               first change or hit on another entry -- from every chunk's record; the
//               members before the cut finish (verdicts, policy counters, metrics) and
//               their updates of e are summarised as a function of the three bits e has
//               when the chunk starts (the 8-state transition table of hot_fold, and per
//               starting state the reductions: the lifetime class of the last update that
//               set one, the flags seen and whether any ran, per direction), with the
//               counter sums;
//  k_ct_hot     per elephant: the chunk summaries composed in order -- (T1, R1) then
//               (T2, R2) = (T2 . T1, R1 then R2 evaluated at T1(x)) -- applied to e once,
//               then the walk resumes at the cut, serially as before.
// An elephant of established packets is one round of parallel lookups instead of a chain
// of ~24-us chunks.
#ifndef CV_HPAR_MIN
#define CV_HPAR_MIN (8 * 1024)
#endif
constexpr uint32_t HPAR_RUNS = 256, HPAR_MIN = CV_HPAR_MIN;
// g.hot layout: per run r < HPAR_RUNS: HP_RUN + 4r {off, cnt, first chunk, chunks} (chunks
// 0: not in parallel), HP_CUT + 4r {cut, e lo, e hi, -}; HP_TOTAL the chunks; per chunk q:
// HP_CHUNK + 8q {run, first change, first hit, hit on another entry, e lo, e hi, -, -} and
// hp_sum + 16q its summary {T, R[8], pk[2], by[2], -}, R[x] = valid | class << 1 |
// any tx << 3 | any rx << 4 | seen tx << 8 | seen rx << 16
constexpr uint32_t HP_RUN = 0, HP_CUT = 4 * HPAR_RUNS, HP_TOTAL = 8 * HPAR_RUNS, HP_CHUNK = 8 * HPAR_RUNS + 64;
__host__ __device__ constexpr uint32_t hp_sum(uint32_t chunks_cap) { return HP_CHUNK + 8 * chunks_cap; }
__host__ __device__ constexpr uint32_t hp_words(uint32_t chunks_cap) { return hp_sum(chunks_cap) + 16 * chunks_cap; }

__global__ void __launch_bounds__(HOTB) k_hpar_look(DpParams p, BatchDev b, GroupScratch g)
{
    __shared__ unsigned long long fs;
    __shared__ uint32_t fl[4], wsum[17], tot_s;
    // the plan (every workgroup; the first writes it for k_hpar_fin and k_ct_hot)
    {
        const uint32_t nhot = hot_runs(g, Q_NETDEV), r = threadIdx.x;
        uint32_t off = 0, cnt = 0, nch = 0;
        if (r < HPAR_RUNS && r < nhot) {
            off = g.work[r];
            if (off < 2u * g.lim) {
                cnt = g.order[off];
                if (!run_ok(g, off, cnt)) cnt = 0;
            }
            if (cnt >= HPAR_MIN) nch = (cnt + HOTB - 1) / HOTB;
        }
        uint32_t total;
        const uint32_t first = block_excl_scan(nch, wsum, total);
        if (threadIdx.x == 0) tot_s = total <= g.hot_chunks ? total : 0u;   // (past the scratch: all serial)
        __syncthreads();
        if (!tot_s) nch = 0;
        if (blockIdx.x == 0 && r < HPAR_RUNS) {
            uint32_t *run = g.hot + HP_RUN + 4 * r;
            run[0] = off; run[1] = cnt; run[2] = first; run[3] = nch;
            if (r == 0) g.hot[HP_TOTAL] = tot_s;
        }
        __syncthreads();
    }
    const uint32_t total = tot_s;
    for (uint32_t q = blockIdx.x; q < total; q += gridDim.x) {    // (block-uniform) a workgroup per chunk
        // (the plan: recomputed here; block 0's copy is read by the later kernels)
        uint32_t r = 0, off = 0, cnt = 0, first = 0;
        {
            const uint32_t nhot = hot_runs(g, Q_NETDEV);
            uint32_t acc = 0;
            for (uint32_t x = 0; x < HPAR_RUNS && x < nhot; ++x) {   // (uniform; HPAR_RUNS reads, cached)
                const uint32_t o2 = g.work[x];
                if (o2 >= 2u * g.lim) continue;
                const uint32_t c2 = g.order[o2];
                if (c2 < HPAR_MIN || c2 >= 2u * g.lim - o2) continue;
                const uint32_t n2 = (c2 + HOTB - 1) / HOTB;
                if (q < acc + n2) { r = x; off = o2; cnt = c2; first = acc; break; }
                acc += n2;
            }
        }
        (void)r;
        const uint32_t k = (q - first) * HOTB + threadIdx.x;
        const uint32_t x0 = g.order[off + 1];
        if (!pkt_ok(g, x0)) continue;                             // (block-uniform; reported)
        const HashTable ct = ep_netdev4<false>(p, g.srec[2 * x0 + 1].z & 0xFFFFu).ct4;
        HotMember h;
        Acct a{0, 0, nullptr};
        a.ctu = ct_unit(p);
        hot_lookup(p, b, g, ct, off, cnt, k, h, a);
        if (threadIdx.x < 3) fl[threadIdx.x] = cnt;
        __syncthreads();
        if (h.change) atomicMin(&fl[0], k);
        if (h.hr.slot >= 0) atomicMin(&fl[1], k);
        __syncthreads();
        if (h.hr.slot >= 0 && k == fl[1]) fs = (unsigned long long)h.hr.slot;
        __syncthreads();
        if (h.hr.slot >= 0 && (unsigned long long)h.hr.slot != fs) atomicMin(&fl[2], k);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t *rec = g.hot + HP_CHUNK + 8 * q;
            rec[0] = r; rec[1] = fl[0]; rec[2] = fl[1]; rec[3] = fl[2];
            rec[4] = fl[1] < cnt ? (uint32_t)fs : 0u; rec[5] = fl[1] < cnt ? (uint32_t)(fs >> 32) : 0u;
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(HOTB) k_hpar_fin(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    __shared__ HotLds L;
    __shared__ uint32_t R[8], last[8], sums[4], cq[2];
    __shared__ unsigned long long es;
    using M = MetT<false>;
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    const uint32_t total = g.hot[HP_TOTAL];
    for (uint32_t q = blockIdx.x; q < total; q += gridDim.x) {    // (block-uniform) a workgroup per chunk
        const uint32_t r = g.hot[HP_CHUNK + 8 * q];
        const uint32_t off = g.hot[HP_RUN + 4 * r], cnt = g.hot[HP_RUN + 4 * r + 1];
        const uint32_t first = g.hot[HP_RUN + 4 * r + 2], nch = g.hot[HP_RUN + 4 * r + 3];
        // the run's entry (the first chunk with a hit: its first hit's) and its cut
        if (threadIdx.x == 0) { cq[0] = ~0u; cq[1] = cnt; }
        __syncthreads();
        for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x)
            if (g.hot[HP_CHUNK + 8 * (first + c) + 2] < cnt) atomicMin(&cq[0], c);
        __syncthreads();
        if (threadIdx.x == 0)
            es = cq[0] == ~0u ? ~0ull : (unsigned long long)g.hot[HP_CHUNK + 8 * (first + cq[0]) + 5] << 32 |
                                            g.hot[HP_CHUNK + 8 * (first + cq[0]) + 4];
        __syncthreads();
        const unsigned long long e = es;
        for (uint32_t c = threadIdx.x; c < nch; c += blockDim.x) {
            const uint32_t *rec = g.hot + HP_CHUNK + 8 * (first + c);
            uint32_t cut = min(rec[1], rec[3]);
            if (rec[2] < cnt && ((unsigned long long)rec[5] << 32 | rec[4]) != e) cut = min(cut, rec[2]);
            if (cut < cnt) atomicMin(&cq[1], cut);
        }
        __syncthreads();
        const uint32_t cut = cq[1], k0 = (q - first) * HOTB;
        if (q == first && threadIdx.x == 0) {
            uint32_t *c = g.hot + HP_CUT + 4 * r;
            c[0] = cut; c[1] = (uint32_t)e; c[2] = (uint32_t)(e >> 32);
        }
        uint32_t *sum = g.hot + hp_sum(g.hot_chunks) + 16 * q;
        if (k0 >= cut) {                                          // (block-uniform) past the cut: no summary
            if (threadIdx.x < 16) sum[threadIdx.x] = threadIdx.x == 0 ? FX_IDENT : 0u;
            __syncthreads();
            continue;
        }
        const uint32_t x0 = g.order[off + 1];
        if (!pkt_ok(g, x0)) continue;                             // (block-uniform; reported)
        const HashTable ct = ep_netdev4<false>(p, g.srec[2 * x0 + 1].z & 0xFFFFu).ct4;
        HotMember h;
        Acct a{0, 0, m.pc};
        a.ctu = ct_unit(p);
        const uint32_t k = k0 + threadIdx.x;
        hot_lookup(p, b, g, ct, off, cnt, k, h, a);
        const bool fin = h.live && k < cut;
        if (fin) hot_member_finish(p, o, h, a, m, now);
        // the summary of the chunk's updates of e, per starting state x
        const bool part = fin && h.hr.slot >= 0 && (unsigned long long)h.hr.slot == e;
        uint32_t T = FX_IDENT;
        if (part) {
            T = 0;
#pragma unroll
            for (uint32_t x = 0; x < 8; ++x) T |= hit_fx(x, h.hr.action, h.hr.dir, h.hr.tcp, h.hr.seen).x << (3 * x);
        }
        if (threadIdx.x < 8) { R[threadIdx.x] = 0; last[threadIdx.x] = 0; }
        if (threadIdx.x < 4) sums[threadIdx.x] = 0;
        uint32_t tot;
        const uint32_t pre = fx_scan(T, L, &tot);                // (ends with a barrier)
        const int d = h.hr.dir == CT_INGRESS ? 1 : 0;
#pragma unroll 1
        for (uint32_t x = 0; x < 8; ++x) {
            uint32_t lst = 0, bits = 0;
            if (part) {
                const HitFx f = hit_fx(fx_at(pre, x), h.hr.action, h.hr.dir, h.hr.tcp, h.hr.seen);
                if (f.any) {
                    lst = (threadIdx.x + 1) << 8 | (f.life == CT_LIFETIME_TCP ? 1u : f.life == CT_CLOSE_TIMEOUT ? 2u : 0u);
                    bits = (1u << (3 + d)) | (h.hr.seen & 0xFFu) << (d ? 16 : 8);
                }
            }
#pragma unroll
            for (int s2 = 32; s2; s2 >>= 1) {
                lst = max(lst, (uint32_t)__shfl_xor((int)lst, s2, 64));
                bits |= (uint32_t)__shfl_xor((int)bits, s2, 64);
            }
            if ((threadIdx.x & 63) == 0) {
                if (lst) atomicMax(&last[x], lst);
                if (bits) atomicOr(&R[x], bits);
            }
        }
        uint32_t pk[2] = {0u, 0u}, by[2] = {0u, 0u};
        if (part && (p.flags & F_CT_ACCOUNTING)) { pk[d] = 1u; by[d] = h.hr.len; }
#pragma unroll
        for (int s2 = 32; s2; s2 >>= 1)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd) {
                pk[dd] += (uint32_t)__shfl_xor((int)pk[dd], s2, 64);
                by[dd] += (uint32_t)__shfl_xor((int)by[dd], s2, 64);
            }
        if ((threadIdx.x & 63) == 0)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd) {
                if (pk[dd]) atomicAdd(&sums[dd], pk[dd]);
                if (by[dd]) atomicAdd(&sums[2 + dd], by[dd]);
            }
        __syncthreads();
        if (threadIdx.x < 16) {
            uint32_t v = 0;
            if (threadIdx.x == 0) v = tot;
            else if (threadIdx.x <= 8) {
                const uint32_t x = threadIdx.x - 1;
                v = R[x] | (last[x] ? 1u | (last[x] & 3u) << 1 : 0u);
            } else if (threadIdx.x <= 12) v = sums[threadIdx.x - 9];
            sum[threadIdx.x] = v;
        }
        __syncthreads();
    }
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// the elephant r's chunk summaries composed in order and applied to its entry: the whole
// workgroup stages HPF_BATCH summaries at a time in LDS (one round of loads each), thread
// 0 composes them; returns where k_ct_hot resumes (every thread)
constexpr uint32_t HPF_BATCH = 256;
struct HparLds {
    uint32_t sm[HPF_BATCH * 16];
    uint32_t T, A[8], cut;
    unsigned long long pk[2], by[2];
};

__device__ uint32_t hpar_fold(const DpParams &p, const GroupScratch &g, const HashTable &ct, uint32_t r, uint32_t now,
                              HparLds &F)
{
    const uint32_t first = g.hot[HP_RUN + 4 * r + 2], nch = g.hot[HP_RUN + 4 * r + 3];
    if (!nch) return 0;                                           // (block-uniform)
    const uint32_t cut = g.hot[HP_CUT + 4 * r];
    const unsigned long long e = (unsigned long long)g.hot[HP_CUT + 4 * r + 2] << 32 | g.hot[HP_CUT + 4 * r + 1];
    if (e == ~0ull || !cut) return cut;                           // (no hit before the cut)
    const uint32_t used = min(nch, (cut + HOTB - 1) / HOTB);      // chunks with members before the cut
    if (threadIdx.x == 0) {                                       // per starting state: what the updates so far did
        F.T = FX_IDENT;
        for (int x = 0; x < 8; ++x) F.A[x] = 0;
        F.pk[0] = F.pk[1] = F.by[0] = F.by[1] = 0;
    }
    for (uint32_t q0 = 0; q0 < used; q0 += HPF_BATCH) {           // (block-uniform)
        const uint32_t nb = min(HPF_BATCH, used - q0);
        const uint32_t *src = g.hot + hp_sum(g.hot_chunks) + 16 * (first + q0);
        __syncthreads();
        for (uint32_t w = threadIdx.x; w < nb * 16; w += blockDim.x) F.sm[w] = src[w];
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t T = F.T, A[8];
            for (int x = 0; x < 8; ++x) A[x] = F.A[x];
            for (uint32_t q = 0; q < nb; ++q) {
                const uint32_t *sm = F.sm + 16 * q;
                for (uint32_t x = 0; x < 8; ++x) {
                    const uint32_t bx = sm[1 + fx_at(T, x)];
                    if (bx & 1u) A[x] = (A[x] & ~7u) | (bx & 7u);     // (the later update's lifetime class)
                    A[x] |= bx & 0xFFFF18u;                           // (any / seen accumulate)
                }
                T = fx_then(T, sm[0]);
                for (int d = 0; d < 2; ++d) { F.pk[d] += sm[9 + d]; F.by[d] += sm[11 + d]; }
            }
            F.T = T;
            for (int x = 0; x < 8; ++x) F.A[x] = A[x];
        }
    }
    if (threadIdx.x == 0) {
        const int64_t slot = (int64_t)e;
        CtE en;
        ct_load_hot<Ct4Spec>(ct, slot, en);
        uint32_t h[CT_HOTW] = {en.w[8], en.w[9], en.w[10], en.w[11], en.w[12], en.w[13], en.w[0], en.w[2], en.w[4],
                               en.w[6]};
        const uint32_t x0 = bits_x(h[1] & 0xFFFFu), a = F.A[x0];
        const uint32_t seen[2] = {(a >> 8) & 0xFFu, (a >> 16) & 0xFFu}, any[2] = {(a >> 3) & 1u, (a >> 4) & 1u};
        hot_store(ct, slot, h, fx_at(F.T, x0), a & 1u, (a >> 1) & 3u, seen, any, F.pk, F.by, now, p.flags);
    }
    return cut;
}

__global__ void __launch_bounds__(HOTB) k_ct_hot(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    __shared__ HotLds L;
    __shared__ HparLds F;
    using M = MetT<false>;
    M m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    const uint32_t nhot = hot_runs(g, Q_NETDEV);
    for (uint32_t r = blockIdx.x; r < nhot; r += gridDim.x) {     // a workgroup per run
        const uint32_t off = g.work[r];
        if (off >= 2u * g.lim) { if (threadIdx.x == 0) group_err(g, GERR_INDEX); continue; }   // (block-uniform)
        const uint32_t cnt = g.order[off], x0 = g.order[off + 1];
        if (!run_ok(g, off, cnt) || !pkt_ok(g, x0)) continue;
        const HashTable ct = ep_netdev4<false>(p, g.srec[2 * x0 + 1].z & 0xFFFFu).ct4;   // (the run's map)
        // an elephant's members before its cut ran in parallel (k_hpar_*): their updates of
        // its entry folded here, then the walk resumes at the cut
        const uint32_t start = r < HPAR_RUNS ? hpar_fold(p, g, ct, r, now, F) : 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        l1_inv();
        __syncthreads();
        for (uint32_t k0 = start; k0 < cnt;) {                    // (block-uniform)
            // 1. the lookups against the chunk's starting table, read only
            HotMember h;
            Acct a{0, 0, m.pc};
            a.ctu = ct_unit(p);
            hot_lookup(p, b, g, ct, off, cnt, k0 + threadIdx.x, h, a);
            if (threadIdx.x == 0) { L.c = HOTB; L.lead = HOTB; }
            __syncthreads();
            if (h.change) atomicMin(&L.c, threadIdx.x);
            __syncthreads();
            // at most HOT_ENTRIES entries per chunk (the fold runs a pass per entry): the
            // chunk ends at the first hit on a further one -- a hot pair carrying many port
            // flows takes several chunks instead of a pass per flow (advisor r04)
            bool seen_e = !(h.hr.slot >= 0 && threadIdx.x < L.c);
            for (uint32_t ne = 0;; ++ne) {                        // (block-uniform)
                if (threadIdx.x == 0) L.lead = HOTB;
                __syncthreads();
                if (!seen_e) atomicMin(&L.lead, threadIdx.x);
                __syncthreads();
                const uint32_t ld = L.lead;
                if (ld >= HOTB) break;
                if (ne == HOT_ENTRIES) {                          // ld: the first hit on one entry too many
                    if (threadIdx.x == 0) L.c = ld;
                    __syncthreads();
                    break;
                }
                if (threadIdx.x == ld) L.slot = (unsigned long long)h.hr.slot;
                __syncthreads();
                if (!seen_e && (unsigned long long)h.hr.slot == L.slot) seen_e = true;
            }
            if (threadIdx.x == 0) L.lead = HOTB;
            __syncthreads();
            if (h.hr.slot >= 0) atomicMin(&L.lead, threadIdx.x);  // the first hit
            __syncthreads();
            const uint32_t c = L.c;
            uint32_t lead = L.lead;
            if (lead < c && threadIdx.x == lead) {                // its entry, while the others finish
                L.slot = (unsigned long long)h.hr.slot;
                hot_load<Ct4Spec>(ct, L, h.hr.slot);
            }
            // 2. the members before c, in parallel
            if (h.live && threadIdx.x < c) hot_member_finish(p, o, h, a, m, now);
            // 3. their hits' entry updates, entry by entry, in member order
            bool pend = h.live && threadIdx.x < c && h.hr.slot >= 0;
            for (bool first = true; lead < c; first = false) {    // (block-uniform)
                __syncthreads();
                const bool part = pend && (unsigned long long)h.hr.slot == L.slot;
                hot_fold<Ct4Spec>(ct, L, part, h.hr, now, p.flags, first);   // (ends with a barrier)
                pend &= !part;
                if (threadIdx.x == 0) L.lead = HOTB;
                __syncthreads();
                if (pend) atomicMin(&L.lead, threadIdx.x);
                __syncthreads();
                lead = L.lead;
                if (lead < c && threadIdx.x == lead) L.slot = (unsigned long long)h.hr.slot;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // (the entries written before any re-read)
            l1_inv();
            __syncthreads();
            if (c >= HOTB) {                                      // (block-uniform) no member changes a key
                k0 += HOTB;
                continue;
            }
            // 4. member c whole: its create or delete, against the table the fold left
            if (threadIdx.x == c) {
                Acct a1{(h.s1.y >> 16) & 0xFFu, h.s1.y >> 24, m.pc};
                uint8_t ct1 = CT_NONE;
                uint16_t proxy = 0;
                int32_t reason = 0;
                const int rv = handle_policy4<M, false>(p, h.ep, h.s, h.s1.w, (h.s1.z >> 16) & 1u, (h.s1.z >> 17) & 1u,
                                                        now, ct1, proxy, reason, a1, m);
                if (o.ret) o.ret[h.x] = rv;
                if (o.reason) o.reason[h.x] = reason;
                if (o.ct) o.ct[h.x] = ct1;
                if (o.proxy) o.proxy[h.x] = proxy;
                store_out(o, h.x, a1);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            l1_inv();
            __syncthreads();
            k0 += c + 1;
        }
    }
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// stage 2: conntrack + policy, each address-pair group by one lane in packet order (the
// hot runs by k_ct_hot when `hot`)
template <bool EV>
__global__ void __launch_bounds__(BLOCK) CV_NS_OCC k_ct_stage(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now,
                                                    int hot)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    MetT<EV> m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    for_each_run(g, Q_NETDEV, false, [&](uint32_t x, uint32_t n) {
        if (x - p.win_lo < p.win_span) stage2_one(p, b, o, g, x, now, m, n == 1);     // (admission windows)
    }, hot ? hot_runs(g, Q_NETDEV) : 0u);
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// stage 2 of an IPv6 packet: ipv6_local_delivery's tail call into the endpoint's
// handle_policy -> tail_ipv6_policy -> ipv6_policy (bpf_lxc.c:721-862, 1003-1038)
template <class M>
__device__ __forceinline__ void stage2_one6(const DpParams &p, const BatchDev &b, const OutDev &o,
                                            const GroupScratch &g, uint32_t i, uint32_t now, M &m, bool single)
{
    Rec6 r;
    rec_load(r, b, i, b.stride >= 128 ? 8 : (int)(b.stride >> 4));
    const uint4 s1 = g.srec[2 * i + 1];
    const uint32_t meta = s1.z;
    const EpDev ep = G(p.eps)[meta & 0xFFFFu];
    Acct a{(s1.y >> 16) & 0xFFu, s1.y >> 24, m.pc};
    a.ctu = ct_unit(p);
    uint8_t ct = CT_NONE;
    uint16_t proxy = 0;
    int32_t reason = 0;
    Skb6 s = skb6_from(r);
    int64_t lslot = -1;                                          // the destination's cilium_lxc slot
    if constexpr (M::EV) {
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        lslot = (int32_t)g.ifx[i];
    }
    RevNat6Out rn;
    rn.valid = false;
    if (p.budget) a.budget = p.budget[i];
    bool defer = single && !p.ct_guard && !M::EV && a.budget >= 2;
    const int ret = handle_policy6<M, false>(p, ep, s, s1.w, (meta >> 16) & 1u,
                                   ifindex_of(m, p.lxc6, lslot, ((meta >> 17) & 1u) << 17), now, ct, proxy, reason,
                                   a, m, &rn, &defer);
    if (defer) g.gslot[i] = proxy ? COMMIT6 - COMMIT_PROXY : COMMIT6;
    if (M::EV && o.frames && (ret == TC_ACT_OK || ret == TC_ACT_REDIRECT) && !proxy) {
        // ipv6_local_delivery's ipv6_l3, then ipv6_policy's rev-NAT index zeroing and reverse NAT
        const uint8_t *in = b.frames + (size_t)i * b.stride;
        Frame6 f;
        frame6_init(f, r, s.l4off, s.nexthdr, in);
        uint32_t mac[2], nmac[2];
        lxc_macs(p.lxc6, lslot, mac, nmac);
        frame6_l3(f, nmac, mac);
        frame6_zero_revnat(f);
        if (rn.valid) frame6_revnat(f, rn);
        frame6_emit(f, in, o.frames + (size_t)i * b.stride, b.stride);
    }
    if (o.ret) o.ret[i] = ret;
    if (o.reason) o.reason[i] = reason;
    if (o.ct) o.ct[i] = ct;
    if (o.proxy) o.proxy[i] = proxy;
    store_out(o, i, a);
}

template <bool EV>
__global__ void __launch_bounds__(BLOCK) k_ct_stage6(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    MetT<EV> m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
    for_each_run(g, Q_NETDEV6, false, [&](uint32_t x, uint32_t n) {
        if (x - p.win_lo < p.win_span) stage2_one6(p, b, o, g, x, now, m, n == 1);
    });
    met_flush(m, p.metrics);
    pol_cache_flush(pc);
}

// The creates of singleton groups, deferred by stage 2 (marked in g.gslot): no other
// packet of the batch can touch the new entry or its ICMP twin (their address pair is
// the group key), so writing them after the stage equals writing them in place, and
// the stage's waves no longer wait on the insert chain of their few creating lanes.
// ct_create4 / ct_create6 (conntrack.h:663-744 / 589-639) with the tuple ct_lookup
// left (ct_l4's tuple reversed: both directions missed) and the ipv{4,6}_policy state.
// A block gathers the marked packets of a span of COMMIT_SPAN packets into LDS (a
// ballot and one LDS atomic per wave) and then creates them with every lane busy:
// about one packet in seven carries a create, and a lane-per-packet pass would keep
// six lanes of seven idle while the seventh walks its insert chains.
//
// A deferred create cannot fail on capacity (launches that could reach max_entries
// run guarded and do not defer) and fails on the probe limit only when CT_MAX_PROBE
// consecutive buckets hold live entries (cv_hash.hpp).  Should one fail anyway, the
// packet's outcome is rewritten to the reference's: ipv{4,6}_policy returns
// DROP_CT_CREATE_FAILED, tail_ipv{4,6}_policy sends the drop notification
// (bpf_lxc.c:946-949, 985-990) -- the forward metric the stage counted (a proxy
// redirect counts none) moves to the drop reason; the entries written before the
// failing one stay, as in the reference.
constexpr uint32_t COMMIT_SPAN = BLOCK * 8;
__device__ __forceinline__ int commit_one(const DpParams &p, const BatchDev &b, const GroupScratch &g, uint32_t i,
                                          bool v6, uint32_t now, Acct &a, uint32_t &len)
{
    const uint4 s1 = g.srec[2 * i + 1];
    uint32_t seen;
    if (!v6) {
        const EpDev ep = ep_netdev4<false>(p, s1.z & 0xFFFFu);
        const Skb4 s = skb4_unpack(g.srec[2 * i], s1.x, s1.y & 0x3FFu, b.stride);
        Tuple4 t;
        t.nexthdr = s.nexthdr;
        t.daddr = s.daddr;
        t.saddr = s.saddr;
        t.dport = t.sport = 0;
        ct_l4<false>(t, s.h, CT_INGRESS, seen);
        t.reverse();
        len = s.len;
        const CtState sn{0, 0, 0, 0, 0, s1.w};
        return ct_create<false>(ep.ct4, t, s.len, CT_INGRESS, sn, now, a, false, false, true);
    } else {
        Rec6 r;
        rec_load(r, b, i, b.stride >= 128 ? 8 : (int)(b.stride >> 4));
        const Skb6 s = skb6_from(r);
        Tuple6 t;
#pragma unroll
        for (int j = 0; j < 4; ++j) { t.daddr[j] = s.daddr[j]; t.saddr[j] = s.saddr[j]; }
        t.nexthdr = s.nexthdr;
        t.dport = t.sport = 0;
        ct_l4<true>(t, s.h, CT_INGRESS, seen);
        t.reverse();
        len = s.len;
        const CtState sn{s.daddr[3] & 0xFFFFu, 0, 0, 0, 0, s1.w};
        return ct_create<true>(G(p.eps)[s1.z & 0xFFFFu].ct6, t, s.len, CT_INGRESS, sn, now, a, false, false, true);
    }
}

__device__ __noinline__ void commit_failed(const DpParams &p, const OutDev &o, uint32_t i, uint32_t len, bool proxied)
{
    if (o.ret) o.ret[i] = TC_ACT_SHOT;
    if (o.reason) o.reason[i] = DROP_CT_CREATE_FAILED;
    if (o.proxy) o.proxy[i] = 0;
    if (!p.metrics) return;
    const uint32_t r = (uint8_t)(-DROP_CT_CREATE_FAILED);
    atomicAdd(&p.metrics[(r * 4 + METRIC_INGRESS) * 2], 1ull);
    atomicAdd(&p.metrics[(r * 4 + METRIC_INGRESS) * 2 + 1], (unsigned long long)len);
    if (!proxied) {
        atomicAdd(&p.metrics[(0 * 4 + METRIC_INGRESS) * 2], ~0ull);
        atomicAdd(&p.metrics[(0 * 4 + METRIC_INGRESS) * 2 + 1], 0ull - len);
    }
}

__global__ void __launch_bounds__(BLOCK) k_ct_commit(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsPolicy pc;
    __shared__ uint32_t list[COMMIT_SPAN], lcount;
    pol_cache_init(pc);
    Acct a{0, 0, &pc};
    a.ctu = ct_unit(p);
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * COMMIT_SPAN; base < b.n; base += gridDim.x * COMMIT_SPAN) {
        if (threadIdx.x == 0) lcount = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < COMMIT_SPAN / BLOCK; ++u) {
            const uint32_t i = base + u * BLOCK + threadIdx.x;
            const uint32_t mk = i < b.n && i - p.win_lo < p.win_span ? g.gslot[i] : NONE;
            const bool want = mk >= COMMIT6 - COMMIT_PROXY && mk <= COMMIT4;
            const unsigned long long w = __ballot(want);
            if (!w) continue;
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(&lcount, (uint32_t)__popcll(w));
            at = __shfl(at, 0, 64);
            const uint32_t v6 = (mk == COMMIT6 || mk == COMMIT6 - COMMIT_PROXY) ? 0x80000000u : 0u;
            const uint32_t px = mk <= COMMIT4 - COMMIT_PROXY ? 0x40000000u : 0u;
            if (want) list[at + __popcll(w & ((1ull << lane) - 1))] = i | v6 | px;
        }
        __syncthreads();
        const uint32_t cnt = lcount;
        for (uint32_t k = threadIdx.x; k < cnt; k += BLOCK) {
            const uint32_t e = list[k], i = e & 0x3FFFFFFFu;
            uint32_t len;
            if (commit_one(p, b, g, i, e >> 31, now, a, len) == DROP_CT_CREATE_FAILED)
                commit_failed(p, o, i, len, (e >> 30) & 1u);
        }
        __syncthreads();                                          // (list / lcount reuse)
    }
    __syncthreads();
    pol_cache_flush(pc);
}

// ------------------------------------------------------------------ binned grouping
// The netdev path groups its packets by (CT map, address pair) without an atomic per
// packet: k_netdev_front writes each staged packet's 64-bit key (0: not staged);
// k_gkey_hist counts the keys per (bin = the key's top gbits bits, binning block) in
// LDS; three small kernels scan the counts into offsets; k_gkey_scatter writes every
// staged packet as {packet, key low word} into its bin's slice; k_gbin_group sorts each
// bin by (key low word, packet) in LDS -- a bin past LCAP entries by sub-bins, and a
// hot address pair's members by packet through a bitmap (gbin_split_key) -- so a
// group's members end up contiguous and in packet order, and writes the runs {size,
// members} into `order`; k_heads_count / k_heads_place list the groups' first
// packets in packet order, size class by size class (the
// `work` and `single` lists for_each_run reads).  Keys that share the bin bits and the
// low word merge into one group (about 2^-32 per pair of groups in a bin): a coarser
// grouping, equally exact.
// Measured against the node-table join it replaced (one CAS per packet into a 128 MiB
// table at the device's atomic rate, then list walks to flatten the groups): DESIGN.md §5.
constexpr uint32_t SCAN_TILE = 4096;                             // entries per scan block (1024 x 4)
constexpr uint32_t LCAP = 2048;                                  // bin entries sorted in LDS
constexpr uint32_t GUNROLL = 8;                                  // keys loaded ahead per thread

__device__ __forceinline__ uint32_t gkey_bin(unsigned long long k, uint32_t bits)
{
    return (uint32_t)(k >> (64 - bits));
}

// exclusive scan of one value per thread over a block of up to 1024 threads
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, uint32_t &total)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t w = 0; w < nw; ++w) { const uint32_t t = wsum[w]; wsum[w] = acc; acc += t; }
        wsum[16] = acc;
    }
    __syncthreads();
    total = wsum[16];
    const uint32_t r = wsum[wv] + incl - v;
    __syncthreads();                                              // (wsum reuse)
    return r;
}

__global__ void __launch_bounds__(1024) k_gkey_hist(GroupScratch g, uint32_t n)
{
    extern __shared__ uint32_t hist[];                           // one counter per bin
    const uint32_t nb = 1u << g.gbits;
    if (blockIdx.x == 0 && threadIdx.x == 0) {                   // (this grouping's split keys and big bins:
        g.cursor[SJOB_WORD] = 0;                                  //  none yet; a launch may run two groupings)
        g.cursor[BIG_WORD] = 0;
    }
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) hist[j] = 0;
    __syncthreads();
    const uint32_t tile = (n + GBLK - 1) / GBLK, lo = blockIdx.x * tile, hi = min(n, lo + tile);
    // GUNROLL keys in flight per thread (one block per CU: a load per iteration left
    // the kernel latency-bound)
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += GUNROLL * blockDim.x) {
        unsigned long long k[GUNROLL];
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            k[u] = i < hi ? __builtin_nontemporal_load(&g.pkey[i]) : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u)
            if (k[u]) atomicAdd(&hist[gkey_bin(k[u], g.gbits)], 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) g.gcnt[j * GBLK + blockIdx.x] = hist[j];
}

// Scan of L u32 values in place (the bin-major counts here, the admission prefixes
// below): tile sums (SCAN_TILE values per block), their exclusive scan (+ the total)
// by one block, then each tile scanned with its offset, exclusive or inclusive.
__global__ void __launch_bounds__(1024) k_scan_tiles(const uint32_t *c, uint32_t L, uint32_t *tsum)
{
    __shared__ uint32_t wsum[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; ++k) v += j + k < L ? c[j + k] : 0u;
    uint32_t total;
    block_excl_scan(v, wsum, total);
    if (threadIdx.x == 0) tsum[blockIdx.x] = total;
}

__global__ void __launch_bounds__(1024) k_scan_top(uint32_t *tsum, uint32_t tiles, uint32_t *total_out)
{
    __shared__ uint32_t wsum[17];
    uint32_t v[4], sum = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t t = threadIdx.x * 4 + k;
        v[k] = t < tiles ? tsum[t] : 0u;
        sum += v[k];
    }
    uint32_t total;
    uint32_t e = block_excl_scan(sum, wsum, total);
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t t = threadIdx.x * 4 + k;
        if (t < tiles) tsum[t] = e;
        e += v[k];
    }
    if (threadIdx.x == 0 && total_out) *total_out = total;
}

__global__ void __launch_bounds__(1024) k_scan_apply(uint32_t *c, uint32_t L, const uint32_t *tsum, int inclusive)
{
    __shared__ uint32_t wsum[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    uint32_t v[4], sum = 0;
    for (uint32_t k = 0; k < 4; ++k) { v[k] = j + k < L ? c[j + k] : 0u; sum += v[k]; }
    uint32_t total;
    uint32_t e = block_excl_scan(sum, wsum, total) + tsum[blockIdx.x];
    for (uint32_t k = 0; k < 4; ++k) {
        if (j + k < L) c[j + k] = inclusive ? e + v[k] : e;
        e += v[k];
    }
}

// in-place scan of c[0, L) (L <= SCAN_TILE * 4096); tsum: ceil(L / SCAN_TILE) words
void launch_scan(uint32_t *c, uint32_t L, uint32_t *tsum, uint32_t *total_out, bool inclusive, hipStream_t s)
{
    const uint32_t tiles = (L + SCAN_TILE - 1) / SCAN_TILE;
    if (!tiles) return;
    hipLaunchKernelGGL(k_scan_tiles, dim3(tiles), dim3(1024), 0, s, c, L, tsum);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, tsum, tiles, total_out);
    hipLaunchKernelGGL(k_scan_apply, dim3(tiles), dim3(1024), 0, s, c, L, tsum, inclusive ? 1 : 0);
}

__global__ void __launch_bounds__(1024) k_gkey_scatter(GroupScratch g, uint32_t n)
{
    extern __shared__ uint32_t pos[];                            // the block's next slot per bin
    const uint32_t nb = 1u << g.gbits;
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) pos[j] = g.gcnt[j * GBLK + blockIdx.x];
    __syncthreads();
    const uint32_t tile = (n + GBLK - 1) / GBLK, lo = blockIdx.x * tile, hi = min(n, lo + tile);
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += GUNROLL * blockDim.x) {
        unsigned long long k[GUNROLL];
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const uint32_t i = i0 + u * blockDim.x;
            k[u] = i < hi ? __builtin_nontemporal_load(&g.pkey[i]) : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            if (!k[u]) continue;
            const uint32_t at = atomicAdd(&pos[gkey_bin(k[u], g.gbits)], 1u);
            g.gent[at] = make_uint2(i0 + u * blockDim.x, (uint32_t)k[u]);
        }
    }
}

// ascending bitonic sort of v[0, p), p a power of two, by the block's threads
template <class P>
__device__ __forceinline__ void bitonic_sort(P v, uint32_t p)
{
    for (uint32_t k = 2; k <= p; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < p / 2; t += blockDim.x) {
                const uint32_t i = 2 * j * (t / j) + (t % j), l = i + j;
                const unsigned long long a = v[i], b = v[l];
                if ((a > b) == ((i & k) == 0)) { v[i] = b; v[l] = a; }
            }
            __syncthreads();
        }
}

constexpr uint32_t SUBMAX = 48;                                  // largest sub-bin sorted by insertion
constexpr uint32_t SPLIT_PAR = 4096;                              // split keys ordered by k_gbin_tiles from here
__device__ __forceinline__ uint32_t sub_of(unsigned long long composite) { return (uint32_t)(composite >> 34) & 255u; }

// base[idx] += 1 for the active lanes, returning each its old value, with one LDS atomic
// for all the lanes that share the first active lane's counter: a bin or tile of a hot
// address pair sends nearly every lane to one counter, which plain LDS atomics serialise
__device__ __forceinline__ uint32_t lds_inc(uint32_t *base, uint32_t idx, bool active)
{
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long act = __ballot(active);
    if (!act) return 0;
    const int l = __ffsll((long long)act) - 1;
    const uint32_t li = (uint32_t)__shfl((int)idx, l, 64);
    const unsigned long long same = __ballot(active && idx == li);
    uint32_t b = 0;
    if (lane == (uint32_t)l) b = atomicAdd(&base[li], (uint32_t)__popcll(same));
    b = (uint32_t)__shfl((int)b, l, 64);
    if ((same >> lane) & 1ull) return b + (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
    return active ? atomicAdd(&base[idx], 1u) : 0u;
}

struct GbinLds {                                                  // k_gbin_group's LDS
    unsigned long long lv[LCAP];                                  // (a split key's tile bitmap when not sorting)
    uint16_t perm[LCAP];
    uint32_t sub_cnt[256], sub_off[256], sub_max, wsum[17], fill, big[2];
    uint32_t bcnt[256], boff[256], bfill[256];                    // a bin past LCAP: its sub-bins
    uint32_t pcnt[256], poff[256];                                // a split key: its members per scatter tile
    uint32_t rest, mcount, key, head[NPOS], mused;
};

// v[0, nb) (nb <= LCAP) sorted by composite in LDS: a counting sort by 8 more key bits
// (sub-bins of a few entries), then every entry ranked within its sub-bin by its own
// thread (a rank sort: m compares per entry, all entries at once; one insertion sort per
// sub-bin and thread spent m^2 steps on its largest sub-bin); a sub-bin past SUBMAX takes
// the bitonic sort instead
__device__ void gbin_lds_sort(GbinLds &L, uint32_t nb)
{
    unsigned long long *lv = L.lv;
    uint32_t p = 64;
    while (p < nb) p <<= 1;
    for (uint32_t j = nb + threadIdx.x; j < p; j += blockDim.x) lv[j] = ~0ull;
    uint32_t *cnt = L.sub_cnt, *off = L.sub_off;
    cnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) L.sub_max = 0;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) atomicAdd(&cnt[sub_of(lv[j])], 1u);
    __syncthreads();
    uint32_t total;
    const uint32_t mine = cnt[threadIdx.x];
    off[threadIdx.x] = block_excl_scan(mine, L.wsum, total);
    atomicMax(&L.sub_max, mine);
    cnt[threadIdx.x] = 0;                                         // (reused as the fill counters)
    __syncthreads();
    if (L.sub_max > SUBMAX) {
        bitonic_sort(lv, p);
        return;
    }
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
        const uint32_t sb = sub_of(lv[j]);
        L.perm[off[sb] + atomicAdd(&cnt[sb], 1u)] = (uint16_t)j;
    }
    __syncthreads();
    uint32_t dst[LCAP / 256];
    unsigned long long val[LCAP / 256];
#pragma unroll
    for (uint32_t k = 0; k < LCAP / 256; ++k) {
        const uint32_t j = threadIdx.x + k * 256;
        if (j < nb) {
            const unsigned long long xv = lv[j];
            const uint32_t sb = sub_of(xv), o = off[sb], c = cnt[sb];
            uint32_t rank = 0;
            for (uint32_t q = o; q < o + c; ++q) rank += lv[L.perm[q]] < xv ? 1u : 0u;   // (composites differ)
            dst[k] = o + rank;
            val[k] = xv;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < LCAP / 256; ++k) {
        const uint32_t j = threadIdx.x + k * 256;
        if (j < nb) lv[dst[k]] = val[k];
    }
    __syncthreads();
}

// the first packets of a group of c members: its `hword` marks (and, from NPOS members
// on for position lists, or from 2 members on for runs, its run at `off` in `order`)
__device__ __forceinline__ void gbin_mark(const GroupScratch &g, uint32_t key, uint32_t c, uint32_t off,
                                          const uint32_t *first, uint32_t *big)
{
    const uint32_t q6 = key & 1u;
    if (c > 8) atomicMax(&big[q6], c);
    if (g.flat) {
        // member t < NPOS - 1 on list t; a group past NPOS - 1 members continues as a run
        // on lists NPOS - 1 .. 15 by the size class of what is left of it, so a wave of the
        // continuation launch takes runs of about one length (for_each_at)
        const uint32_t m = c < NPOS ? c : NPOS;
        for (uint32_t t = 0; t < m; ++t) {
            uint32_t list = t;
            if (t + 1 == NPOS) {
                const uint32_t sc = (uint32_t)size_class(c - (NPOS - 1));
                list = NPOS - 1 + (sc < 16 - NPOS ? sc : 16 - NPOS);
            }
            g.hword[first[t]] = (1u + q6 * 16 + list) << 26 | (t + 1 == NPOS ? off : 0u);
        }
        return;
    }
    const uint32_t list = c > 1 ? 15 - (uint32_t)size_class(c) : 15u;   // 15: singletons (bit 25: a singleton)
    g.hword[first[0]] = (1u + q6 * 16 + list) << 26 | (c > 1 ? off : 1u << 25);
}

// one pass over the sorted v[0, nb): the runs into the bin's own region of `order` (2
// words per entry: a run of c members takes c + 1 <= 2c; no allocation atomics), and
// every group's first packet marked with its list and run (k_heads_place lists them in
// packet order)
__device__ void gbin_emit(const GroupScratch &g, GbinLds &L, const unsigned long long *v, uint32_t nb, uint32_t start)
{
    for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
        const uint32_t key = (uint32_t)(v[j] >> 32);
        if (j && (uint32_t)(v[j - 1] >> 32) == key) continue;     // not a group's first member
        uint32_t c = 1;
        while (j + c < nb && (uint32_t)(v[j + c] >> 32) == key) ++c;
        uint32_t off = 0, first[NPOS];
        if (c >= (g.flat ? NPOS : 2u)) {                          // (position lists: the continuation list)
            off = 2 * start + atomicAdd(&L.fill, c + 1);
            uint32_t *o = g.order + off;
            o[0] = c;
            for (uint32_t t = 0; t < c; ++t) o[1 + t] = (uint32_t)v[j + t];
        }
        for (uint32_t t = 0; t < NPOS && t < c; ++t) first[t] = (uint32_t)v[j + t];
        gbin_mark(g, key, c, off, first, L.big);
    }
}

// A sub-bin past LCAP entries (an elephant: one address pair carrying thousands of the
// launch's packets) at r[0, cnt): the key most of 64 samples hold is taken out, its members
// ordered by packet with a bitmap in LDS per scatter tile -- k_gkey_scatter writes a tile's
// entries in any order, but the tiles in packet order -- and written as one run; the
// rest stays at r[0, L.rest) for the next key.  Members past the bitmap go through m.
__device__ void gbin_split_key(const GroupScratch &g, GbinLds &L, unsigned long long *r, uint32_t cnt,
                               uint32_t *m, uint32_t start, uint32_t tile)
{
    __syncthreads();                                              // (every thread has read the last call's rest)
    // the key: the most frequent of 64 evenly spaced samples (wave 0)
    if (threadIdx.x < 64) {
        const uint32_t sk = (uint32_t)(r[(unsigned long long)threadIdx.x * cnt / 64] >> 32);
        uint32_t same = 0;
        for (int l = 0; l < 64; ++l) same += __shfl(sk, l, 64) == sk ? 1u : 0u;
        uint32_t best = same << 6 | (63u - threadIdx.x);          // (ties: the lowest lane)
        for (int d = 32; d; d >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, d, 64));
        if (threadIdx.x == 63u - (best & 63u)) L.key = sk;
    }
    L.pcnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) { L.rest = 0; L.mcount = 0; }
    __syncthreads();
    const uint32_t key = L.key;
    m += L.mused;                                                 // (past the bin's earlier split keys)
    for (uint32_t j0 = 0; j0 < cnt; j0 += GUNROLL * blockDim.x) { // its members per scatter tile
        unsigned long long xs[GUNROLL];                           // (GUNROLL loads in flight: one block
#pragma unroll                                                    //  streams the whole hot bin)
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const uint32_t j = j0 + u * blockDim.x + threadIdx.x;
            xs[u] = j < cnt ? r[j] : ~0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const bool mine = (uint32_t)(xs[u] >> 32) == key && xs[u] != ~0ull;
            lds_inc(L.pcnt, mine ? (uint32_t)xs[u] / tile : 0u, mine);
        }
    }
    __syncthreads();
    uint32_t total;
    L.poff[threadIdx.x] = block_excl_scan(L.pcnt[threadIdx.x], L.wsum, total);
    L.bfill[threadIdx.x] = 0;
    __syncthreads();
    // members to m by tile; the others packed to the front of r (a chunk is read whole
    // before any of it is overwritten: the write position never passes the read one)
    for (uint32_t j0 = 0; j0 < cnt; j0 += GUNROLL * blockDim.x) {
        unsigned long long xs[GUNROLL];
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const uint32_t j = j0 + u * blockDim.x + threadIdx.x;
            xs[u] = j < cnt ? r[j] : ~0ull;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < GUNROLL; ++u) {
            const unsigned long long x = xs[u];
            const bool live = x != ~0ull, mine = live && (uint32_t)(x >> 32) == key, other = live && !mine;
            const uint32_t t = mine ? (uint32_t)x / tile : 0u;
            const uint32_t at = lds_inc(L.bfill, t, mine);
            if (mine) m[L.poff[t] + at] = (uint32_t)x;
            const uint32_t ro = lds_inc(&L.rest, 0u, other);
            if (other) r[ro] = x;
        }
    }
    __syncthreads();
    // the run: a large one is ordered tile by tile in parallel by k_gbin_tiles (a job: the
    // key, its members per tile in m, where the run goes; the next key's members go past
    // these in m), a smaller one here -- per tile the members' bits set in LDS, then read
    // back in order
    const uint32_t c = total;
    const bool listed = c >= (g.flat ? NPOS : 2u);                // (a run in `order`; its offset may be 0)
    if (threadIdx.x == 0) {
        L.mcount = listed ? 2 * start + atomicAdd(&L.fill, c + 1) : 0u;
        const uint32_t jx = c >= SPLIT_PAR ? atomicAdd(&g.cursor[SJOB_WORD], 1u) : ~0u;
        L.head[0] = jx < g.sjob_cap ? jx : ~0u;                   // (the job's index; full: ordered here)
    }
    __syncthreads();
    if (L.head[0] != ~0u) {                                       // (block-uniform)
        uint32_t *job = g.sjob + (size_t)L.head[0] * SJOB_WORDS;
        if (threadIdx.x == 0) {
            job[0] = key;
            job[1] = c;
            job[2] = L.mcount;
            job[3] = listed ? 1u : 0u;
            job[4] = (uint32_t)(m - reinterpret_cast<uint32_t *>(g.gbig));
            job[5] = (uint32_t)tile;
        }
        job[SJOB_PCNT + threadIdx.x] = L.pcnt[threadIdx.x];
        job[SJOB_PCNT + 256 + threadIdx.x] = L.poff[threadIdx.x];
        __syncthreads();
        if (threadIdx.x == 0) L.mused += c;
        __syncthreads();
        return;
    }
    const uint32_t off = L.mcount;
    uint32_t *o = g.order + off;
    if (threadIdx.x == 0 && listed) o[0] = c;
    uint32_t *bm = reinterpret_cast<uint32_t *>(L.lv);            // tile bits (tile <= 2^16: 8 KiB)
    constexpr uint32_t BMW = 2048;
    for (uint32_t t = 0; t < GBLK; ++t) {
        const uint32_t pc = L.pcnt[t], po = L.poff[t];            // (block-uniform)
        if (!pc) continue;
        for (uint32_t w = threadIdx.x; w < BMW; w += blockDim.x) bm[w] = 0;
        __syncthreads();
        const uint32_t base = t * tile;
        for (uint32_t q = threadIdx.x; q < pc; q += blockDim.x) {
            const uint32_t d = m[po + q] - base;
            atomicOr(&bm[d >> 5], 1u << (d & 31));
        }
        __syncthreads();
        constexpr uint32_t PER = BMW / 256;                       // words per thread, in order
        uint32_t wv[PER], n1 = 0;
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) { wv[k] = bm[threadIdx.x * PER + k]; n1 += __popc(wv[k]); }
        uint32_t tot;
        uint32_t rank = po + block_excl_scan(n1, L.wsum, tot);
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k)
            for (uint32_t w = wv[k]; w; w &= w - 1) {
                const uint32_t x = base + (threadIdx.x * PER + k) * 32 + (uint32_t)__ffs((int)w) - 1;
                if (listed) o[1 + rank] = x;
                if (rank < NPOS) L.head[rank] = x;
                ++rank;
            }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        gbin_mark(g, key, c, off, L.head, L.big);
        L.mused += c;
    }
    __syncthreads();
}


// k_gbin_group's split keys, ordered: a workgroup per (job, scatter tile) -- the tile's
// members' bits set in an LDS bitmap (a tile is a contiguous packet range of at most 2^16),
// read back in order into the run at their rank (the tile's offset + the rank within it);
// the members of rank < NPOS are the group's first packets (k_gbin_marks)
__global__ void __launch_bounds__(256) k_gbin_tiles(GroupScratch g)
{
    __shared__ uint32_t bm[2048], wsum[17];
    const uint32_t jobs = min(g.cursor[SJOB_WORD], g.sjob_cap);
    for (uint32_t w = blockIdx.x; w < jobs * GBLK; w += gridDim.x) {   // (block-uniform)
        const uint32_t *job = g.sjob + (size_t)(w / GBLK) * SJOB_WORDS;
        const uint32_t t = w % GBLK, pc = job[SJOB_PCNT + t], po = job[SJOB_PCNT + 256 + t];
        if (!pc) continue;
        const uint32_t *m = reinterpret_cast<const uint32_t *>(g.gbig) + job[4];
        const uint32_t tile = job[5], base = t * tile;
        uint32_t *o = g.order + job[2];
        const bool listed = job[3] != 0;
        for (uint32_t k = threadIdx.x; k < 2048; k += blockDim.x) bm[k] = 0;
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < pc; q += blockDim.x) {
            const uint32_t d = m[po + q] - base;
            if (d < 65536u) atomicOr(&bm[d >> 5], 1u << (d & 31));
        }
        __syncthreads();
        constexpr uint32_t PER = 2048 / 256;                      // words per thread, in order
        uint32_t wv[PER], n1 = 0;
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) { wv[k] = bm[threadIdx.x * PER + k]; n1 += __popc(wv[k]); }
        uint32_t tot;
        uint32_t rank = po + block_excl_scan(n1, wsum, tot);
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k)
            for (uint32_t v = wv[k]; v; v &= v - 1) {
                const uint32_t x = base + (threadIdx.x * PER + k) * 32 + (uint32_t)__ffs((int)v) - 1;
                if (!pkt_ok(g, x) || rank >= job[1]) { ++rank; continue; }   // (a corrupt job)
                if (listed) o[1 + rank] = x;
                if (rank < NPOS) const_cast<uint32_t *>(job)[SJOB_HEAD + rank] = x;
                ++rank;
            }
        __syncthreads();
    }
}

// every split key's group marks (its first packets, from k_gbin_tiles), one thread per job
__global__ void __launch_bounds__(256) k_gbin_marks(GroupScratch g)
{
    const uint32_t jobs = min(g.cursor[SJOB_WORD], g.sjob_cap);
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < jobs; w += gridDim.x * blockDim.x) {
        const uint32_t *job = g.sjob + (size_t)w * SJOB_WORDS;
        const uint32_t key = job[0], c = job[1];
        bool ok = run_ok(g, job[2], c);
        for (uint32_t t = 0; t < NPOS && t < c; ++t) ok = ok && pkt_ok(g, job[SJOB_HEAD + t]);
        if (!ok) continue;                                        // (a corrupt job: reported, skipped)
        if (job[3]) g.order[job[2]] = c;
        uint32_t big[2] = {0u, 0u};
        gbin_mark(g, key, c, job[2], job + SJOB_HEAD, big);
        if (big[key & 1u]) atomicMax(&g.cursor[GMAX_WORD0 + ((key & 1u) ? g.q6 : g.q4)], big[key & 1u]);
    }
}

// Big bins in parallel.  A bin of BIG_MIN entries or more is an elephant's (one address
// pair carrying a large share of the launch) next to a few ordinary keys: one workgroup
// streaming it (the sub-bin scatter, then gbin_split_key's two passes) took 5 ms for
// 837 000 entries.  Four launches take its dominant key out across the device first:
// k_gbig_list picks the key (the most frequent of 64 evenly spaced samples, as
// gbin_split_key does) and opens a record; k_gbig_count counts the key's members per
// scatter tile and the other entries, a workgroup per chunk of the bin; k_gbig_plan
// turns a key with at least half of its bin into a split-key job (its run first in the
// bin's region of `order`, its members per tile at the tile offsets); k_gbig_place writes
// the members by tile and packs the other entries to the front of the bin's gbig region.
// k_gbin_group then groups only those others, and k_gbin_tiles orders the job's members.
constexpr uint32_t BIG_CHUNK = 2048;                              // bin entries per workgroup step (256 x 8)

__device__ __forceinline__ void gbin_range(const GroupScratch &g, uint32_t b, uint32_t &start, uint32_t &nb)
{
    const uint32_t nbins = 1u << g.gbits, m = nbins * GBLK;
    start = g.gcnt[b * GBLK];
    nb = (b + 1 < nbins ? g.gcnt[(b + 1) * GBLK] : g.gcnt[m]) - start;
}

// a wave per bin: its record, or 0
__global__ void __launch_bounds__(256) k_gbig_list(GroupScratch g)
{
    const uint32_t lane = threadIdx.x & 63, b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= (1u << g.gbits) || !g.gbx) return;                 // (wave-uniform)
    uint32_t start, nb;
    gbin_range(g, b, start, nb);
    uint32_t *bx = g.gbx;
    if (nb < BIG_MIN) {
        if (!lane) bx[b] = 0;
        return;
    }
    const uint32_t sk = g.gent[start + (uint32_t)((unsigned long long)lane * nb / 64)].y;
    uint32_t same = 0;
    for (int l = 0; l < 64; ++l) same += __shfl(sk, l, 64) == sk ? 1u : 0u;
    uint32_t best = same << 6 | (63u - lane);                     // (ties: the lowest lane)
    for (int d = 32; d; d >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, d, 64));
    const uint32_t key = __shfl(sk, 63 - (int)(best & 63u), 64);
    uint32_t r = 0;
    if (!lane) r = atomicAdd(&g.cursor[BIG_WORD], 1u);
    r = (uint32_t)__shfl((int)r, 0, 64);
    if (r >= g.gbx_cap) {                                         // (full: the bin stays whole)
        if (!lane) bx[b] = 0;
        return;
    }
    uint32_t *rec = bx + GBIN_MAX + (size_t)r * BIGW;
    if (!lane) {
        rec[0] = b; rec[1] = key; rec[2] = start; rec[3] = nb;
        rec[4] = 0; rec[5] = 0; rec[6] = ~0u; rec[7] = 0;
        bx[b] = r + 1;
    }
    for (uint32_t t = lane; t < 2 * GBLK; t += 64) rec[BIG_PCNT + t] = 0;
}

// the records' chunks over the grid: record k's chunk u goes to workgroup (u + 97 k) mod grid
template <class F>
__device__ __forceinline__ void for_each_big_chunk(const GroupScratch &g, F &&fn)
{
    const uint32_t nrec = g.gbx ? min(g.cursor[BIG_WORD], g.gbx_cap) : 0u;
    for (uint32_t k = 0; k < nrec; ++k) {                         // (block-uniform)
        uint32_t *rec = g.gbx + GBIN_MAX + (size_t)k * BIGW;
        const uint32_t nb = rec[3], chunks = (nb + BIG_CHUNK - 1) / BIG_CHUNK;
        const uint32_t u0 = (blockIdx.x + gridDim.x - (97u * k) % gridDim.x) % gridDim.x;
        for (uint32_t u = u0; u < chunks; u += gridDim.x) fn(rec, u);
    }
}

__global__ void __launch_bounds__(256) k_gbig_count(GroupScratch g, uint32_t n)
{
    __shared__ uint32_t cnt[GBLK], other;
    const uint32_t tile = (n + GBLK - 1) / GBLK;
    for_each_big_chunk(g, [&](uint32_t *rec, uint32_t u) {
        const uint32_t key = rec[1], start = rec[2], nb = rec[3];
        cnt[threadIdx.x] = 0;
        if (!threadIdx.x) other = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t v = 0; v < BIG_CHUNK / 256; ++v) {
            const uint32_t j = u * BIG_CHUNK + v * 256 + threadIdx.x;
            const bool live = j < nb;
            const uint2 e = live ? g.gent[start + j] : make_uint2(0u, 0u);
            const bool mine = live && e.y == key;
            lds_inc(cnt, mine ? min(e.x / tile, GBLK - 1) : 0u, mine);
            lds_inc(&other, 0u, live && !mine);
        }
        __syncthreads();
        if (cnt[threadIdx.x]) atomicAdd(&rec[BIG_PCNT + threadIdx.x], cnt[threadIdx.x]);
        if (!threadIdx.x && other) atomicAdd(&rec[5], other);
        __syncthreads();
    });
}

// a workgroup per record: a key with half of its bin or more becomes a split-key job
__global__ void __launch_bounds__(256) k_gbig_plan(GroupScratch g, uint32_t n)
{
    __shared__ uint32_t wsum[17], jx;
    const uint32_t nrec = g.gbx ? min(g.cursor[BIG_WORD], g.gbx_cap) : 0u;
    if (blockIdx.x >= nrec) return;
    uint32_t *rec = g.gbx + GBIN_MAX + (size_t)blockIdx.x * BIGW;
    const uint32_t pc = rec[BIG_PCNT + threadIdx.x];
    uint32_t c;
    const uint32_t po = block_excl_scan(pc, wsum, c);
    const uint32_t start = rec[2], nb = rec[3];
    if (!threadIdx.x) {
        jx = ~0u;
        if (2 * c >= nb && c + rec[5] == nb) {                    // (the others fit before the sub-bins)
            const uint32_t j = atomicAdd(&g.cursor[SJOB_WORD], 1u);
            if (j < g.sjob_cap) jx = j;
        }
        rec[4] = c;
        rec[6] = jx;
        if (jx == ~0u) g.gbx[rec[0]] = 0;                         // (the bin stays whole)
    }
    __syncthreads();
    if (jx == ~0u) return;
    uint32_t *job = g.sjob + (size_t)jx * SJOB_WORDS;
    rec[BIG_FILL + threadIdx.x] = po;
    job[SJOB_PCNT + threadIdx.x] = pc;
    job[SJOB_PCNT + 256 + threadIdx.x] = po;
    if (!threadIdx.x) {
        job[0] = rec[1];
        job[1] = c;
        job[2] = 2 * start;                                       // (the bin's region of `order`: the run first)
        job[3] = c >= (g.flat ? NPOS : 2u) ? 1u : 0u;
        job[4] = 4 * start + 2 * nb;                              // (the members: gbin's `mem` of the bin)
        job[5] = (n + GBLK - 1) / GBLK;
    }
}

__global__ void __launch_bounds__(256) k_gbig_place(GroupScratch g, uint32_t n)
{
    __shared__ uint32_t cnt[GBLK], base[GBLK], other, obase;
    const uint32_t tile = (n + GBLK - 1) / GBLK;
    for_each_big_chunk(g, [&](uint32_t *rec, uint32_t u) {
        if (rec[6] == ~0u) return;                                // (block-uniform: not taken out)
        const uint32_t key = rec[1], start = rec[2], nb = rec[3];
        uint32_t *mem = reinterpret_cast<uint32_t *>(g.gbig + 2 * (size_t)start + nb);
        uint2 *rest = reinterpret_cast<uint2 *>(g.gbig + 2 * (size_t)start);
        uint2 es[BIG_CHUNK / 256];
        cnt[threadIdx.x] = 0;
        if (!threadIdx.x) other = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t v = 0; v < BIG_CHUNK / 256; ++v) {
            const uint32_t j = u * BIG_CHUNK + v * 256 + threadIdx.x;
            const bool live = j < nb;
            es[v] = live ? g.gent[start + j] : make_uint2(0u, 0u);
            const bool mine = live && es[v].y == key;
            lds_inc(cnt, mine ? min(es[v].x / tile, GBLK - 1) : 0u, mine);
            lds_inc(&other, 0u, live && !mine);
        }
        __syncthreads();
        base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&rec[BIG_FILL + threadIdx.x], cnt[threadIdx.x]) : 0u;
        cnt[threadIdx.x] = 0;
        if (!threadIdx.x) {
            obase = other ? atomicAdd(&rec[7], other) : 0u;
            other = 0;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t v = 0; v < BIG_CHUNK / 256; ++v) {
            const uint32_t j = u * BIG_CHUNK + v * 256 + threadIdx.x;
            const bool live = j < nb, mine = live && es[v].y == key;
            const uint32_t t = mine ? min(es[v].x / tile, GBLK - 1) : 0u;
            const uint32_t at = lds_inc(cnt, t, mine);
            const uint32_t ro = lds_inc(&other, 0u, live && !mine);
            if (mine) mem[base[t] + at] = es[v].x;
            else if (live) rest[obase + ro] = es[v];
        }
        __syncthreads();
    });
}

__global__ void __launch_bounds__(256) k_gbin_group(GroupScratch g, uint32_t n)
{
    __shared__ GbinLds L;
    const uint32_t b = blockIdx.x;
    uint32_t start, nb0;
    gbin_range(g, b, start, nb0);
    if (!nb0) return;                                             // (block-uniform)
    // a big bin whose dominant key k_gbig_* took out: its other entries, packed at the front
    // of its gbig region, after the key's run in `order` and its members in `mem`
    const uint32_t bx = g.gbx ? g.gbx[b] : 0u;
    const uint32_t *rec = bx ? g.gbx + GBIN_MAX + (size_t)(bx - 1) * BIGW : nullptr;
    const uint32_t taken = rec ? rec[4] : 0u, nb = rec ? rec[5] : nb0;
    const uint2 *src = rec ? reinterpret_cast<const uint2 *>(g.gbig + 2 * (size_t)start) : g.gent + start;
    if (threadIdx.x == 0) { L.fill = rec ? taken + 1 : 0u; L.mused = taken; }
    if (threadIdx.x < 2) L.big[threadIdx.x] = 0;
    // composite {key low word, packet}: sorted, a group's members are contiguous and ascending
    if (nb <= LCAP) {
        for (uint32_t j = threadIdx.x; j < nb; j += blockDim.x) {
            const uint2 e = src[j];
            L.lv[j] = (unsigned long long)e.y << 32 | e.x;
        }
        __syncthreads();
        if (nb) {
            gbin_lds_sort(L, nb);
            gbin_emit(g, L, L.lv, nb, start);
        }
    } else {
        // a bin past LCAP: its entries by 8 more key bits into sub-bins (gbig: 2 words per
        // entry, the second half the split keys' member lists), sub-bins of up to LCAP
        // sorted in LDS a batch at a time, a larger one split key by key
        unsigned long long *gv = g.gbig + 2 * (size_t)start + (rec ? nb : 0u);   // (past the packed others)
        uint32_t *mem = reinterpret_cast<uint32_t *>(g.gbig + 2 * (size_t)start + nb0);
        const uint32_t tile = (n + GBLK - 1) / GBLK;
        L.bcnt[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < nb; j0 += GUNROLL * blockDim.x) {
            uint2 es[GUNROLL];
#pragma unroll
            for (uint32_t u = 0; u < GUNROLL; ++u) {
                const uint32_t j = j0 + u * blockDim.x + threadIdx.x;
                es[u] = j < nb ? src[j] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < GUNROLL; ++u)
                lds_inc(L.bcnt, sub_of((unsigned long long)es[u].y << 32 | es[u].x),
                        j0 + u * blockDim.x + threadIdx.x < nb);
        }
        __syncthreads();
        uint32_t total;
        L.boff[threadIdx.x] = block_excl_scan(L.bcnt[threadIdx.x], L.wsum, total);
        L.bfill[threadIdx.x] = 0;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < nb; j0 += GUNROLL * blockDim.x) {
            uint2 es[GUNROLL];
#pragma unroll
            for (uint32_t u = 0; u < GUNROLL; ++u) {
                const uint32_t j = j0 + u * blockDim.x + threadIdx.x;
                es[u] = j < nb ? src[j] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (uint32_t u = 0; u < GUNROLL; ++u) {
                const bool live = j0 + u * blockDim.x + threadIdx.x < nb;
                const unsigned long long x = (unsigned long long)es[u].y << 32 | es[u].x;
                const uint32_t sb = sub_of(x);
                const uint32_t at = lds_inc(L.bfill, sb, live);
                if (live) gv[L.boff[sb] + at] = x;
            }
        }
        __syncthreads();
        for (uint32_t sb = 0; sb < 256;) {                        // (block-uniform)
            uint32_t cnt = L.bcnt[sb];
            if (cnt > LCAP) {
                unsigned long long *r = gv + L.boff[sb];
                while (cnt > LCAP) {
                    gbin_split_key(g, L, r, cnt, mem, start, tile);
                    cnt = L.rest;
                }
                for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) L.lv[j] = r[j];
                ++sb;
            } else {
                const uint32_t lo = L.boff[sb];
                cnt = 0;
                while (sb < 256 && cnt + L.bcnt[sb] <= LCAP) cnt += L.bcnt[sb++];
                for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) L.lv[j] = gv[lo + j];
            }
            __syncthreads();
            if (cnt) {
                gbin_lds_sort(L, cnt);
                gbin_emit(g, L, L.lv, cnt, start);
            }
            __syncthreads();
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 && L.big[threadIdx.x])                    // (diagnostics: the largest group)
        atomicMax(&g.cursor[GMAX_WORD0 + (threadIdx.x ? g.q6 : g.q4)], L.big[threadIdx.x]);
}

// The groups' first packets listed in packet order, list by list (IPv4 runs class
// 15 .. 1, IPv4 singletons, the same for IPv6): per tile of HTILE packets a count per
// list, one scan, then each tile places its heads (ranks within a tile by LDS atomics:
// a wave's lanes still take packets of one tile) and the lists' lengths go to the
// cursor words for_each_run reads.  The stage's first members then read their stage
// records and write their verdicts along the batch instead of at random.
constexpr uint32_t HTILE = 4096;
__global__ void __launch_bounds__(1024) k_heads_count(GroupScratch g, uint32_t n, uint32_t tiles)
{
    __shared__ uint32_t c[32];
    if (threadIdx.x < 32) c[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t k = 0; k < HTILE / 1024; ++k) {
        const uint32_t x = blockIdx.x * HTILE + k * 1024 + threadIdx.x;
        const uint32_t h = x < n ? g.hword[x] >> 26 : 0u;
        if (h) atomicAdd(&c[h - 1], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 32) g.hcnt[threadIdx.x * tiles + blockIdx.x] = c[threadIdx.x];
}

__global__ void __launch_bounds__(1024) k_heads_place(GroupScratch g, uint32_t n, uint32_t tiles)
{
    __shared__ uint32_t pos[32], start[4];
    if (threadIdx.x < 32) pos[threadIdx.x] = g.hcnt[threadIdx.x * tiles + blockIdx.x];
    if (threadIdx.x < 4) start[threadIdx.x] = g.hcnt[(threadIdx.x >> 1) * 16 * tiles + (threadIdx.x & 1) * 15 * tiles];
    if (blockIdx.x == 0 && threadIdx.x < 32) {                    // list lengths -> the cursor words
        const uint32_t key = threadIdx.x, q = key >> 4 ? g.q6 : g.q4, list = key & 15u;
        const uint32_t cnt = g.hcnt[(key + 1) * tiles] - g.hcnt[key * tiles];   // ([32 * tiles] = the total)
        if (g.flat) {
            g.cursor[qcls(q, list)] = cnt;                        // position list lengths (for_each_at)
        } else {
            if (list == 15) g.cursor[SINGLE_WORD0 + q] = cnt;
            g.cursor[qcls(q, list == 15 ? 0 : 15 - list)] = cnt;
        }
    }
    __syncthreads();
    for (uint32_t k = 0; k < HTILE / 1024; ++k) {
        const uint32_t x = blockIdx.x * HTILE + k * 1024 + threadIdx.x;
        const uint32_t hw = x < n ? g.hword[x] : 0u, h = hw >> 26;
        if (!h) continue;
        const uint32_t key = h - 1, q6 = key >> 4, at = atomicAdd(&pos[key], 1u);
        if (g.flat) (q6 ? g.work6 : g.work)[at - start[q6 * 2]] = (key & 15u) + 1 >= NPOS ? (hw & ((1u << 25) - 1)) : x;
        else if ((key & 15u) == 15u) (q6 ? g.single6 : g.single)[at - start[q6 * 2 + 1]] = x;
        else (q6 ? g.work6 : g.work)[at - start[q6 * 2]] = hw & ((1u << 25) - 1);
    }
}

// test hook (CV_JOB_INJECT): one split-key job more counted than the grouping wrote, its
// run word past `order` -- the r05 fault's shape (an egress launch's two groupings once
// shared the job count, so the second read the first's jobs); k_gbin_marks must skip it
// and report it (-EPROTO at the context's next call), never index through it
__global__ void k_job_inject(GroupScratch g)
{
    if (threadIdx.x) return;
    const uint32_t j = g.cursor[SJOB_WORD];
    if (j >= g.sjob_cap) return;
    uint32_t *job = g.sjob + (size_t)j * SJOB_WORDS;
    job[0] = 0u;
    job[1] = 2u;
    job[2] = 0xFFFFFFF0u;
    job[3] = 1u;
    g.cursor[SJOB_WORD] = j + 1u;
}

void launch_gbin_groups(const GroupScratch &g, uint32_t n, hipStream_t s)
{
    const uint32_t nb = 1u << g.gbits, m = nb * GBLK;
    hipLaunchKernelGGL(k_gkey_hist, dim3(GBLK), dim3(1024), nb * 4, s, g, n);
    launch_scan(g.gcnt, m, g.gcnt + m + 1, g.gcnt + m, false, s);
    hipLaunchKernelGGL(k_gkey_scatter, dim3(GBLK), dim3(1024), nb * 4, s, g, n);
    hipLaunchKernelGGL(k_gbig_list, dim3((nb + 3) / 4), dim3(256), 0, s, g);   // (big bins: dominant keys out)
    hipLaunchKernelGGL(k_gbig_count, dim3(512), dim3(256), 0, s, g, n);
    hipLaunchKernelGGL(k_gbig_plan, dim3(g.gbx_cap), dim3(256), 0, s, g, n);
    hipLaunchKernelGGL(k_gbig_place, dim3(512), dim3(256), 0, s, g, n);
    hipLaunchKernelGGL(k_gbin_group, dim3(nb), dim3(256), 0, s, g, n);
    hipLaunchKernelGGL(k_gbin_tiles, dim3(1024), dim3(256), 0, s, g);   // (split keys: elephant pairs)
    if (getenv("CV_JOB_INJECT")) hipLaunchKernelGGL(k_job_inject, dim3(1), dim3(64), 0, s, g);
    hipLaunchKernelGGL(k_gbin_marks, dim3(8), dim3(256), 0, s, g);
    const uint32_t tiles = (n + HTILE - 1) / HTILE;
    hipLaunchKernelGGL(k_heads_count, dim3(tiles), dim3(1024), 0, s, g, n, tiles);
    launch_scan(g.hcnt, 32 * tiles, g.hcnt + 32 * tiles + 1, g.hcnt + 32 * tiles, false, s);
    hipLaunchKernelGGL(k_heads_place, dim3(tiles), dim3(1024), 0, s, g, n, tiles);
}

// ------------------------------------------------------------------ CT map API
// Single-element BPF_MAP_{LOOKUP,UPDATE,DELETE}_ELEM on a device-resident CT table
// (the agent side of pkg/maps/ctmap: GC deletes, dumps, restores), with the kernel
// hash map's errnos: NOEXIST on an existing key -EEXIST, EXIST on a missing one
// -ENOENT, a new key past max_entries -E2BIG.  Keeps the live-entry count.
template <class S>
__device__ void ct_op(HashTable t, int op, uint64_t flags, uint32_t *io)
{
    uint32_t key[S::KW];
    for (int j = 0; j < S::KW; ++j) key[j] = io[j];
    uint32_t *val = io + S::KW, *rcp = io + S::KW + 16;
    int rc = 0;
    int64_t s = dev_find<S>(t, key, nullptr);
    if (op == 0) {
        if (s < 0) rc = -ENOENT;
        else {
            CtE e;
            ct_load<S>(t, s, e);
            for (int k = 0; k < 16; ++k) val[k] = e.w[k];
        }
    } else if (op == 1) {
        if (s >= 0 && flags == 1) rc = -EEXIST;
        else if (s < 0 && flags == 2) rc = -ENOENT;
        else if (s < 0 && t.live && *t.live >= t.cap) rc = -E2BIG;
        else {
            bool created;
            s = dev_upsert<S>(t, key, &created);
            if (s < 0) rc = -E2BIG;
            else {
                if (created && t.live) atomicAdd(t.live, 1ull);
                CtE e;
                for (int k = 0; k < 16; ++k) e.w[k] = val[k];
                ct_store<S>(t, s, e);
            }
        }
    } else {
        if (s < 0) rc = -ENOENT;
        else {
            dev_kill<S>(t, s);
            if (t.live) atomicAdd(t.live, ~0ull);
        }
    }
    *rcp = (uint32_t)rc;
}

__global__ void k_ct_op(HashTable t, int v6, int op, uint64_t flags, uint32_t *io)
{
    if (threadIdx.x || blockIdx.x) return;
    if (v6) ct_op<Ct6Spec>(t, op, flags, io);
    else ct_op<Ct4Spec>(t, op, flags, io);
}

// Initial fill of a CT map from the agent's entries (a restore, or a synthetic table):
// n distinct keys (KW words each) and ct_entry values (16 words each), inserted in
// parallel (the CAS slot claim of dev_upsert); *fail counts keys past the probe limit.
template <class S>
__device__ void ct_load_t(HashTable t, const uint32_t *keys, const uint32_t *vals, uint64_t n, uint32_t *fail)
{
    for (uint64_t i = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        uint32_t k[S::KW];
#pragma unroll
        for (int j = 0; j < S::KW; ++j) k[j] = keys[i * S::KW + j];
        bool created;
        const int64_t sl = dev_upsert<S>(t, k, &created);
        if (sl < 0) { atomicAdd(fail, 1u); continue; }
        CtE e;
        const uint4 *q = reinterpret_cast<const uint4 *>(vals + i * 16);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint4 v = q[w];
            e.w[4 * w] = v.x; e.w[4 * w + 1] = v.y; e.w[4 * w + 2] = v.z; e.w[4 * w + 3] = v.w;
        }
        ct_store<S>(t, sl, e, created);
    }
}

__global__ void __launch_bounds__(BLOCK) k_ct_load(HashTable t, int v6, const uint32_t *keys, const uint32_t *vals,
                                                   uint64_t n, uint32_t *fail)
{
    if (v6) ct_load_t<Ct6Spec>(t, keys, vals, n, fail);
    else ct_load_t<Ct4Spec>(t, keys, vals, n, fail);
}

int launch_ct_load(const HashTable &t, int v6, const uint32_t *keys, const uint32_t *vals, uint64_t n, uint32_t *fail,
                   hipStream_t s)
{
    if (!n) return 0;
    uint64_t g = (n + BLOCK - 1) / BLOCK;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_ct_load, dim3((uint32_t)g), dim3(BLOCK), 0, s, t, v6, keys, vals, n, fail);
    return launch_status(__func__);
}

// every live entry (tag >= 3): its slot index, key and value, compacted in no order
// (the host sorts by slot: the table's walk order, stable while entries stay put)
template <class S>
__device__ void ct_scan(HashTable t, uint64_t nslots, uint64_t *slots, uint32_t *keys, uint32_t *vals, uint32_t *count,
                        uint32_t max)
{
    for (uint64_t x = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; x < nslots; x += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t b = x / S::SPB;
        const int sl = (int)(x % S::SPB);
        const uint32_t *bw = t.buckets + b * S::BW;
        const uint32_t tag = (bw[sl >> 2] >> (8 * (sl & 3))) & 0xFFu;
        if (tag < 3) continue;
        const uint32_t at = atomicAdd(count, 1u);
        if (at >= max) continue;
        if (slots) slots[at] = x;
        for (int j = 0; j < S::KW; ++j) keys[(size_t)at * S::KW + j] = bw[S::KEY0 + sl * S::KS + j];
        CtE e;
        ct_load<S>(t, (int64_t)x, e);
        for (int j = 0; j < 16; ++j) vals[(size_t)at * 16 + j] = e.w[j];
    }
}

__global__ void k_ct_scan(HashTable t, int v6, uint64_t nslots, uint64_t *slots, uint32_t *keys, uint32_t *vals,
                          uint32_t *count, uint32_t max)
{
    if (v6) ct_scan<Ct6Spec>(t, nslots, slots, keys, vals, count, max);
    else ct_scan<Ct4Spec>(t, nslots, slots, keys, vals, count, max);
}

// ctmap.GC with GCFilterByTime (pkg/maps/ctmap/ctmap.go:247-448): one pass over the
// table, a lane per bucket: read the 8 tag bytes, then the lifetime word of every
// live slot, and mark the expired ones dead (the bucket's tag word rewritten once;
// the pass runs stream-ordered between batches, so it is the only writer).
//
// Tombstones: a lookup walks past dead slots until a bucket with an empty one, so the
// bucket's dead slots (old deletes and this pass's) become empty again when no probe
// chain needs to pass through bucket b.  Invariant: a live key stored in bucket s with
// home h has no empty slot in [h, s).  If bucket b+1 has an empty slot, no key beyond
// b+1 has its home at or before b+1; if every live key of b+1 also has its home in
// b+1, no key past b has its home at or before b, and b's dead slots may empty.  The
// check reads b+1 while its own lane may change it; those changes only delete keys or
// add empty slots, which keeps the conclusion true (a key read half-deleted looks
// displaced: the bucket then just keeps its tombstones this pass).
// n words at word offset o of a 128-B-aligned bucket set to zero, 16 B at a time where
// aligned (o and n are compile-time constants here: the branches fold away)
__device__ __forceinline__ void zero_words(uint32_t *bw, int o, int n)
{
    if ((o & 3) && n >= 2 && !(o & 1)) { *reinterpret_cast<uint2 *>(bw + o) = make_uint2(0u, 0u); o += 2; n -= 2; }
    for (; n >= 4 && !(o & 3); o += 4, n -= 4) *reinterpret_cast<uint4 *>(bw + o) = make_uint4(0u, 0u, 0u, 0u);
    for (; n >= 2 && !(o & 1); o += 2, n -= 2) *reinterpret_cast<uint2 *>(bw + o) = make_uint2(0u, 0u);
    for (; n > 0; ++o, --n) bw[o] = 0u;
}

template <class S>
__device__ void ct_gc(HashTable t, uint64_t nb, uint32_t time, uint32_t *deleted, uint32_t *freed)
{
    uint32_t mine = 0, cleared = 0;
    // GC_U buckets per thread and iteration: their tag words, then the live slots'
    // lifetimes, are loaded before any is used (a scan bound by load latency at one
    // bucket per step)
    constexpr int GC_U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (uint64_t b0 = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; b0 < nb; b0 += GC_U * stride) {
        uint64_t tgs[GC_U];
        uint32_t lifes[GC_U][S::SPB];
#pragma unroll
        for (int u = 0; u < GC_U; ++u) {
            const uint64_t b = b0 + u * stride;
            tgs[u] = 0;
            if (b < nb) {
                const uint2 tg = *reinterpret_cast<const uint2 *>(t.buckets + b * S::BW);
                tgs[u] = (uint64_t)tg.x | ((uint64_t)tg.y << 32);
            }
        }
#pragma unroll
        for (int u = 0; u < GC_U; ++u)
#pragma unroll
            for (int sl = 0; sl < S::SPB; ++sl) {
                const uint64_t b = b0 + u * stride;
                lifes[u][sl] = (b < nb && ((uint32_t)(tgs[u] >> (8 * sl)) & 0xFFu) >= 3)
                                   ? *ct_hot<S>(t, (int64_t)(b * S::SPB + sl)) : 0u;   // lifetime: hot word 0
            }
#pragma unroll
        for (int u = 0; u < GC_U; ++u) {
            const uint64_t b = b0 + u * stride;
            if (b >= nb) break;
            uint32_t *bw = t.buckets + b * S::BW;
            uint64_t tags = tgs[u], out = tags;
            bool dead = false;
#pragma unroll
            for (int sl = 0; sl < S::SPB; ++sl) {
                const uint32_t tag = (uint32_t)(tags >> (8 * sl)) & 0xFFu;
                if (tag == TAG_DEAD) dead = true;
                if (tag < 3) continue;
                const uint32_t life = lifes[u][sl];
                if (life < time) {
                    out = (out & ~(0xFFull << (8 * sl))) | ((uint64_t)TAG_DEAD << (8 * sl));
                    zero_words(bw, S::KEY0 + sl * S::KS, S::KS);   // free slots hold zero keys,
                    uint4 *c = reinterpret_cast<uint4 *>(t.vals + (b * S::SPB + sl) * CT_COLD);   // hot and side words
                    c[0] = c[1] = make_uint4(0, 0, 0, 0);
                    ++mine;
                    dead = true;
                }
            }
            if (dead) {
                const uint64_t nx = (b + 1) & t.mask;
                const uint32_t *nw = t.buckets + nx * S::BW;        // (any version of it will do, above)
                const uint64_t ntags = (uint64_t)nw[0] | ((uint64_t)nw[1] << 32);
                bool has_empty = false, displaced = false;
#pragma unroll
                for (int sl = 0; sl < S::SPB; ++sl) {
                    const uint32_t tag = (uint32_t)(ntags >> (8 * sl)) & 0xFFu;
                    has_empty |= tag == TAG_EMPTY;
                    if (tag < 3) continue;
                    uint32_t key[S::KW], tg2;
#pragma unroll
                    for (int j = 0; j < S::KW; ++j) key[j] = nw[S::KEY0 + sl * S::KS + j];
                    displaced |= (home_hash<S>(key, tg2) & t.mask) != nx;
                }
                if (has_empty && !displaced) {
#pragma unroll
                    for (int sl = 0; sl < S::SPB; ++sl)
                        if (((out >> (8 * sl)) & 0xFFu) == TAG_DEAD) { out &= ~(0xFFull << (8 * sl)); ++cleared; }
                }
            }
            if (out != tags) *reinterpret_cast<uint2 *>(bw) = make_uint2((uint32_t)out, (uint32_t)(out >> 32));
        }
    }
    const unsigned long long fr = wave_sum(cleared);
    if ((threadIdx.x & 63) == 0 && fr && freed) atomicAdd(freed, (uint32_t)fr);
    const unsigned long long tot = wave_sum(mine);
    if ((threadIdx.x & 63) == 0 && tot) {
        atomicAdd(deleted, (uint32_t)tot);
        if (t.live) atomicAdd(t.live, 0ull - tot);
    }
}

__global__ void __launch_bounds__(BLOCK) k_ct_gc(HashTable t, int v6, uint64_t nb, uint32_t time, uint32_t *deleted)
{
    if (v6) ct_gc<Ct6Spec>(t, nb, time, deleted, deleted + 1);
    else ct_gc<Ct4Spec>(t, nb, time, deleted, deleted + 1);
}

// deleted[0]: entries the pass deleted, deleted[1]: tombstones it turned back into empty slots
int launch_ct_gc(const HashTable &t, int v6, uint64_t nb, uint32_t time, uint32_t *deleted, hipStream_t s)
{
    uint64_t g = (nb + BLOCK - 1) / BLOCK;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_ct_gc, dim3((uint32_t)(g ? g : 1)), dim3(BLOCK), 0, s, t, v6, nb, time, deleted);
    return launch_status(__func__);
}

// slots by tag class: out[0] empty, out[1] dead (tombstones), out[2] live
template <class S>
__device__ void ct_tags(HashTable t, uint64_t nb, unsigned long long *out)
{
    uint32_t c[3] = {0, 0, 0};
    for (uint64_t b = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * BLOCK) {
        const uint32_t w = t.buckets[b * S::BW];
#pragma unroll
        for (int sl = 0; sl < S::SPB; ++sl) {
            const uint32_t tag = (w >> (8 * sl)) & 0xFFu;
            c[tag == TAG_EMPTY ? 0 : tag == TAG_DEAD ? 1 : 2]++;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const unsigned long long v = wave_sum(c[k]);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&out[k], v);
    }
}

__global__ void __launch_bounds__(BLOCK) k_ct_tags(HashTable t, int v6, uint64_t nb, unsigned long long *out)
{
    if (v6) ct_tags<Ct6Spec>(t, nb, out);
    else ct_tags<Ct4Spec>(t, nb, out);
}

int launch_ct_tags(const HashTable &t, int v6, uint64_t nb, unsigned long long *out, hipStream_t s)
{
    uint64_t g = (nb + BLOCK - 1) / BLOCK;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_ct_tags, dim3((uint32_t)(g ? g : 1)), dim3(BLOCK), 0, s, t, v6, nb, out);
    return launch_status(__func__);
}

__global__ void __launch_bounds__(BLOCK) k_gather_u64(unsigned long long *const *ptrs, unsigned long long *out,
                                                      uint32_t n)
{
    for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < n; k += gridDim.x * BLOCK)
        out[k] = __hip_atomic_load(ptrs[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int grid_for(uint32_t n);

// ------------------------------------------------------------------ room check (CtBound, cv_dp.hpp)
// per-workgroup sums of the per-map bounds (a popular endpoint's map would take one
// global atomic per packet: Zipf endpoints serialised the check on one word)
constexpr uint32_t BND_SLOTS = 1024, BND_EMPTY = 0xFFFFFFFFu;
struct BoundLds {
    uint32_t key[BND_SLOTS];
    uint32_t cnt[BND_SLOTS];
};

__device__ __forceinline__ void bound_lds_init(BoundLds &l)
{
    for (uint32_t k = threadIdx.x; k < BND_SLOTS; k += blockDim.x) {
        l.key[k] = BND_EMPTY;
        l.cnt[k] = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ void bound_lds_flush(BoundLds &l, const CtBound &bd)
{
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < BND_SLOTS; k += blockDim.x)
        if (l.key[k] != BND_EMPTY && l.cnt[k]) atomicAdd(bd.bound + l.key[k], (unsigned long long)l.cnt[k]);
}

__device__ __forceinline__ void bound_add(const CtBound &bd, BoundLds *l, const uint16_t *epmi, uint32_t e, uint32_t w)
{
    if (e >= bd.n_eps) return;
    const uint32_t m = epmi[e];
    if (m >= bd.nmaps) return;
    if (l) {
        for (uint32_t h = (m * 0x9E3779B1u) >> 22, k = 0; k < 16; ++k, h = (h + 1) & (BND_SLOTS - 1)) {
            const uint32_t old = atomicCAS(&l->key[h], BND_EMPTY, m);
            if (old == BND_EMPTY || old == m) {
                atomicAdd(&l->cnt[h], w);
                return;
            }
        }
    }
    atomicAdd(bd.bound + m, (unsigned long long)w);
}

// the endpoint index (0-based) of a local endpoint address, or ~0 (host / none)
__device__ __forceinline__ uint32_t bound_ep(const DpParams &p, const uint32_t *addr, bool v6)
{
    uint32_t iv = 0;
    const int64_t sl = v6 ? dev_find<LxcV6Spec>(p.lxc6, addr, &iv) : dev_find<LxcV4Spec>(p.lxc4, addr, &iv);
    if (sl < 0 || (iv & (1u << 16)) || !p.ep_of_lxc) return ~0u;
    const uint32_t e = p.ep_of_lxc[iv & 0xFFFFu];
    return e ? e - 1 : ~0u;
}

__device__ __forceinline__ uint32_t bound_ld32(const uint8_t *f) { return f[0] | f[1] << 8 | f[2] << 16 | (uint32_t)f[3] << 24; }

// per packet (or delivery record): its source map's and destination map's creates; the
// service masters that may serve it counted per LB slot
__global__ void __launch_bounds__(BLOCK) k_bound_pkts(DpParams p, BatchDev b, const uint4 *records, CtBound bd)
{
    __shared__ BoundLds lds;
    BoundLds *L = &lds;
    bound_lds_init(lds);
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < b.n; i += gridDim.x * BLOCK) {
        if (bd.mode == 2) {                                       // a delivery record: its destination
            const uint32_t w = reinterpret_cast<const uint32_t *>(records + (size_t)i * DEL_SLOTS)[b.stride >= 128 ? 12 : 6];
            bound_add(bd, L, b.stride >= 128 ? bd.epmi6 : bd.epmi4, w & 0xFFFFu, bd.w_dst);
            continue;
        }
        const uint8_t *f = b.frames + (size_t)i * b.stride;
        const uint32_t len = min(b.len[i], b.stride), eth = f[12] << 8 | f[13];
        const bool v6 = eth == 0x86DDu;
        if ((eth != 0x0800u && !v6) || len < (v6 ? 54u : 34u)) continue;   // (no conntrack)
        if (v6 && b.stride < 128) continue;                       // (E_TRUNC: IPv6 needs 128-B records)
        const uint16_t *epmi = v6 ? bd.epmi6 : bd.epmi4;
        if (bd.mode == 1) bound_add(bd, L, epmi, bd.src_ep ? bd.src_ep[i] : bd.ep0, bd.w_src);
        uint32_t da[4];
        for (int j = 0; j < (v6 ? 4 : 1); ++j) da[j] = bound_ld32(f + (v6 ? 38 : 30) + 4 * j);
        bound_add(bd, L, epmi, bound_ep(p, da, v6), bd.w_dst);
        if (bd.mode != 1) continue;
        // the service masters (daddr, dport) and (daddr, 0) that may serve it (lb{4,6}_lookup_service)
        uint32_t nh, off;
        if (!v6) {
            nh = f[23];
            off = 14 + 4 * (f[14] & 0xFu);
        } else {
            nh = f[20];
            off = 54;
        }
        uint32_t dport = 0;
        if (v6 && nh != 6 && nh != 17 && nh != 58) {              // extension headers: the datapath's own
            Rec6 r;                                               // walk (ipv6_hdrlen, as the front runs it)
            rec_load(r, b, i, 8);
            const int hl = ipv6_hdrlen(r, nh);
            if (hl < 0) continue;                                 // (dropped before any conntrack)
            off = 14 + hl;
            if (nh == 6 || nh == 17) {
                const L4Hdr h = l4_read<54>(r, (int)off);
                if (h.c2b) continue;                              // (dropped: E_FAULT / E_TRUNC)
                dport = h.p2;
            } else if (nh != 58 && nh != 1) {
                continue;                                         // (skip_service_lookup)
            }
        } else if (nh == 6 || nh == 17) {
            if (off + 4 > len) {                                  // (a port the check cannot read)
                atomicAdd(bd.flag + 1, 1u);
                continue;
            }
            dport = f[off + 2] | f[off + 3] << 8;
        } else if (nh != 1 && nh != 58) {
            continue;                                             // (skip_service_lookup)
        }
        for (int k = 0; k < 2; ++k) {
            if (k == 0 && !dport) continue;
            const uint32_t port = k == 0 ? dport : 0u;
            if (!v6) {
                const uint32_t key[2] = {da[0], port};
                uint32_t v[3];
                const int64_t sl = dev_find<Lb4Spec>(p.lb4, key, v);
                if (sl >= 0 && (v[1] >> 16)) atomicAdd(bd.svc4 + sl, 1u);
            } else {
                const uint32_t key[5] = {da[0], da[1], da[2], da[3], port};
                uint32_t v[6];
                const int64_t sl = dev_find<Lb6Spec>(p.lb6, key, v);
                if (sl >= 0 && (v[4] >> 16)) atomicAdd(bd.svc6 + sl, 1u);
            }
        }
    }
    bound_lds_flush(lds, bd);
}

// every backend (slave entry) of a master that may serve packets: its endpoint's map
// takes up to w_dst creates per such packet
template <class S, bool V6>
__global__ void __launch_bounds__(BLOCK) k_bound_svc(DpParams p, CtBound bd)
{
    const HashTable &t = V6 ? p.lb6 : p.lb4;
    const uint32_t *cnt = V6 ? bd.svc6 : bd.svc4;
    const uint64_t slots = (t.mask + 1) * S::SPB;
    for (uint64_t x = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; x < slots; x += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t bk = x / S::SPB;
        const uint32_t sl = (uint32_t)(x % S::SPB);
        const uint32_t *bw = t.buckets + bk * S::BW;
        const uint32_t tag = (bw[sl >> 2] >> (8 * (sl & 3))) & 0xFFu;
        if (tag < 3) continue;
        uint32_t key[S::KW];
        for (int j = 0; j < S::KW; ++j) key[j] = bw[S::KEY0 + sl * S::KS + j];
        if (!(key[S::KW - 1] >> 16)) continue;                   // (a master entry)
        key[S::KW - 1] &= 0xFFFFu;
        uint32_t v[S::IVW];
        const int64_t ms = dev_find<S>(t, key, v);
        if (ms < 0 || !cnt[ms]) continue;
        uint32_t be[4];
        for (int j = 0; j < (V6 ? 4 : 1); ++j) be[j] = bw[S::IVAL0 + sl * S::IVW + j];
        bound_add(bd, nullptr, V6 ? bd.epmi6 : bd.epmi4, bound_ep(p, be, V6), bd.w_dst * cnt[ms]);
    }
}

__global__ void __launch_bounds__(BLOCK) k_bound_check(CtBound bd)
{
    const unsigned long long unseen = (unsigned long long)bd.flag[1] * bd.w_dst;
    for (uint32_t m = blockIdx.x * BLOCK + threadIdx.x; m < bd.nmaps; m += gridDim.x * BLOCK)
        if (*bd.live[m] + bd.bound[m] + unseen > bd.cap[m]) bd.flag[0] = 1u;
}

int launch_ct_bound(const DpParams &p, const BatchDev &b, const uint4 *records, const CtBound &bd, hipStream_t s)
{
    if (b.n) hipLaunchKernelGGL(k_bound_pkts, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, records, bd);
    if (bd.mode == 1) {
        if (p.lb4.buckets) hipLaunchKernelGGL((k_bound_svc<Lb4Spec, false>), dim3(1024), dim3(BLOCK), 0, s, p, bd);
        if (p.lb6.buckets) hipLaunchKernelGGL((k_bound_svc<Lb6Spec, true>), dim3(1024), dim3(BLOCK), 0, s, p, bd);
    }
    hipLaunchKernelGGL(k_bound_check, dim3((bd.nmaps + BLOCK - 1) / BLOCK < 256 ? (bd.nmaps + BLOCK - 1) / BLOCK + 1 : 256),
                       dim3(BLOCK), 0, s, bd);
    return launch_status(__func__);
}

int launch_gather_u64(unsigned long long *const *ptrs, unsigned long long *out, uint32_t n, hipStream_t s)
{
    if (!n) return 0;
    hipLaunchKernelGGL(k_gather_u64, dim3((n + BLOCK - 1) / BLOCK < 1024 ? (n + BLOCK - 1) / BLOCK : 1024), dim3(BLOCK),
                       0, s, ptrs, out, n);
    return launch_status(__func__);
}

// ------------------------------------------------------------------ host launchers
int grid_for(uint32_t n)
{
    uint32_t g = (n + BLOCK - 1) / BLOCK;
    if (g > 2048) g = 2048;
    return g ? (int)g : 1;
}

int launch_xdp_prefilter(const DpParams &p, const BatchDev &b, const OutDev &o, hipStream_t s)
{
    if (!b.n) return 0;
    hipLaunchKernelGGL(k_xdp_prefilter, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o);
    return launch_status(__func__);
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
    return launch_status(__func__);
}

int launch_policy_ingress(const DpParams &p, int ep, const BatchDev &b, const OutDev &o, hipStream_t s)
{
    if (!b.n) return 0;
    const uint32_t grid = (b.n + PPT * BLOCK - 1) / (PPT * BLOCK);
    hipLaunchKernelGGL(k_policy_ingress, dim3(grid), dim3(BLOCK), 0, s, p, ep, b, o);
    return launch_status(__func__);
}

// test hook (CV_LIST_INJECT): the first singleton and the first listed run of the IPv4
// queue name a packet / an `order` offset past the launch, as a stale or corrupt list would
__global__ void k_list_inject(GroupScratch g)
{
    if (threadIdx.x) return;
    if (g.cursor[SINGLE_WORD0 + Q_NETDEV]) g.single[0] = 0xFFFFFFF0u;
    uint32_t multi = 0;
    for (int c = 1; c < NCLASS; ++c) multi += g.cursor[qcls(Q_NETDEV, c)];
    if (multi) g.work[0] = 0xFFFFFFF0u;
}

int launch_netdev_front(const DpParams &p, const BatchDev &b, int with_prefilter, const OutDev &o,
                        const GroupScratch &g0, hipStream_t s)
{
    GroupScratch g = g0;
    g.lim = b.n;
    if (!b.n) return 0;
    const bool ev = o.frames || p.notify || p.trace;              // the instance with the optional outputs
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    if (ev) hipLaunchKernelGGL(k_netdev_front<true>, grid, blk, 0, s, p, b, o, g, with_prefilter);
    else hipLaunchKernelGGL(k_netdev_front<false>, grid, blk, 0, s, p, b, o, g, with_prefilter);
    if (const int r = launch_status(__func__)) return r;
    launch_gbin_groups(g, b.n, s);                                // both families' runs and singletons, listed
    if (getenv("CV_LIST_INJECT")) hipLaunchKernelGGL(k_list_inject, dim3(1), dim3(64), 0, s, g);
    return launch_status(__func__);
}

// the IPv4 runs, then the IPv6 runs (the two families' conntrack state is disjoint, so
// the order between them is free), then the deferred creates
int launch_netdev_stages(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o, const GroupScratch &g0,
                         hipStream_t s)
{
    GroupScratch g = g0;
    g.lim = b.n;
    if (!b.n) return 0;
    const bool ev = o.frames || p.notify || p.trace;
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    // the hot runs by whole waves (plain instance, no admission budgets or guards)
    const int hot = !ev && !p.ct_guard && !p.budget && !getenv("CV_NO_HOT_RUNS");
    if (hot) {                                                    // elephants: their chunks in parallel first
        hipLaunchKernelGGL(k_hpar_look, dim3(1024), dim3(HOTB), 0, s, p, b, g);
        hipLaunchKernelGGL(k_hpar_fin, dim3(1024), dim3(HOTB), 0, s, p, b, o, g, now);
        hipLaunchKernelGGL(k_ct_hot, dim3(512), dim3(HOTB), 0, s, p, b, o, g, now);
    }
    if (ev) hipLaunchKernelGGL(k_ct_stage<true>, grid, blk, 0, s, p, b, o, g, now, 0);
    else hipLaunchKernelGGL(k_ct_stage<false>, grid, blk, 0, s, p, b, o, g, now, hot);
    GroupScratch g6 = g;
    g6.single = g.single6;
    g6.work = g.work6;
    if (ev) hipLaunchKernelGGL(k_ct_stage6<true>, grid, blk, 0, s, p, b, o, g6, now);
    else hipLaunchKernelGGL(k_ct_stage6<false>, grid, blk, 0, s, p, b, o, g6, now);
    if (!p.ct_guard) hipLaunchKernelGGL(k_ct_commit, grid, blk, 0, s, p, b, o, g, now);
    return launch_status(__func__);
}

int launch_netdev_ingress(const DpParams &p, const BatchDev &b, uint32_t now, int with_prefilter, const OutDev &o,
                          const GroupScratch &g, hipStream_t s)
{
    const int r = launch_netdev_front(p, b, with_prefilter, o, g, s);
    return r ? r : launch_netdev_stages(p, b, now, o, g, s);
}

// ------------------------------------------------------------------ conntrack admission
// Next to a CT map's max_entries the batch result depends on the order of creates and
// deletes across groups: the kernel hash map fails an insert of a new key once the
// count is at max_entries (-E2BIG: DROP_CT_CREATE_FAILED) and a delete makes room.  In
// packet order, with r the map's room, a delete makes r + 1 and a packet that tries A
// creates of new entries (its tuple, then its ICMP twin only if the tuple went in)
// gets min(A, r) of them, r - that: a walk reflected at 0, so r after packet j is
// x_j - min(0, min_{q <= j} x_q) with x_j = r_start + the sum of (D - A) up to j --
// two scans.  What each packet creates and deletes comes from k_ct_intent, against
// the table as the window starts: ipv4_policy / ipv6_policy (bpf_lxc.c:865-979,
// 721-849) delete only on CT_ESTABLISHED with a denying verdict and create only on
// CT_NEW with an allowing one, the tuple (absent: the lookup just missed) and the twin
// if it is absent.  A key an earlier member of the packet's group created in this
// window exists iff that member's budget covered it -- a budget the scans compute from
// the intents: k_ct_intent reads the previous pass's budgets and run_admitted repeats
// the pass until no intent changes (a fixed point; the dependencies only point back in
// packet order, so it is the sequential answer, and a pass that changes packet c
// leaves every packet up to c exact).  The stage then runs the window with each
// packet's budget (Acct::budget in ct_put): exactly the sequential run's successes and
// failures, at full width.
// What earlier members of a run did in this window, in packet order: each event a key
// (by hash; a hit is confirmed against the member's key re-derived from its record),
// the member, and its kind: 0 a delete (certain), 1 / 2 a create that went in iff the
// member's budget reaches 1 (its tuple) / 2 (its ICMP twin, tried second).
// Past N events a run's events move to its spill table (a region of Admit::evt
// addressed by the run's place in `order`, 4 slots per member at most half full, slots
// stamped with the pass), which keeps the latest event per key hash -- a run of many
// creates (a busy endpoint's map next to its limit) no longer ends the window.
template <class T>
struct Changed {
    static constexpr int N = 6;
    uint64_t h[N];
    uint32_t ev[N];                                               // member | kind << 30
    int n = 0;
    unsigned long long *tab = nullptr;                            // {hash, stamp << 32 | event} per slot
    uint32_t cap = 0, stamp = 0;
    bool spill = false;
    __device__ void reset() { n = 0; spill = false; tab = nullptr; }
    __device__ bool overflow() const { return n > N && !spill; }
    __device__ void put(uint64_t hk, uint32_t e)
    {
        uint32_t sl = (uint32_t)(hk % cap);
        for (uint32_t k = 0; k < cap; ++k, sl = sl + 1 == cap ? 0u : sl + 1) {
            const unsigned long long w1 = tab[2 * (size_t)sl + 1];
            if ((uint32_t)(w1 >> 32) != stamp || tab[2 * (size_t)sl] == hk) {
                tab[2 * (size_t)sl] = hk;
                tab[2 * (size_t)sl + 1] = (unsigned long long)stamp << 32 | e;
                return;
            }
        }
    }
    __device__ uint32_t find(uint64_t hk) const                   // the latest event on hk, or ~0u
    {
        uint32_t sl = (uint32_t)(hk % cap);
        for (uint32_t k = 0; k < cap; ++k, sl = sl + 1 == cap ? 0u : sl + 1) {
            const unsigned long long w1 = tab[2 * (size_t)sl + 1];
            if ((uint32_t)(w1 >> 32) != stamp) return ~0u;
            if (tab[2 * (size_t)sl] == hk) return (uint32_t)w1;
        }
        return ~0u;
    }
    __device__ void add(const T &t, uint32_t member, uint32_t kind)
    {
        uint32_t k[T::KW];
        t.key(k);
        const uint64_t hk = key_hash<typename T::Spec>(k);
        const uint32_t e = member | kind << 30;
        if (!spill && n == N && tab) {                            // (to the run's table)
            spill = true;
            for (int j = 0; j < N; ++j) put(h[j], ev[j]);
        }
        if (spill) { put(hk, e); return; }
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j == n) { h[j] = hk; ev[j] = e; }
        ++n;
    }
};

// the conntrack tuple packet i looks up in ipv4_policy / ipv6_policy (false: none)
template <bool V6, class T>
__device__ __forceinline__ bool intent_tuple(const DpParams &p, const BatchDev &b, const GroupScratch &g, uint32_t i,
                                             T &t, EpDev &ep, uint32_t &src)
{
    const uint4 s1 = g.srec[2 * i + 1];
    const uint32_t meta = s1.z;
    uint32_t seen;
    src = s1.w;
    if constexpr (!V6) {
        ep = ep_netdev4<false>(p, meta & 0xFFFFu);
        if ((p.flags & F_DROP_ALL) || !ep.ipv4) return false;
        const Skb4 s = skb4_unpack(g.srec[2 * i], s1.x, s1.y & 0x3FFu, b.stride);
        if (s.len < 34) return false;
        t.nexthdr = s.nexthdr; t.daddr = s.daddr; t.saddr = s.saddr; t.dport = t.sport = 0;
        return ct_l4<false>(t, s.h, CT_INGRESS, seen) >= 0;
    } else {
        ep = G(p.eps)[meta & 0xFFFFu];
        if (p.flags & F_DROP_ALL) return false;
        Rec6 r;
        rec_load(r, b, i, b.stride >= 128 ? 8 : (int)(b.stride >> 4));
        const Skb6 s = skb6_from(r);
        if (s.len < 54 || s.l4off < 0) return false;
#pragma unroll
        for (int j = 0; j < 4; ++j) { t.daddr[j] = s.daddr[j]; t.saddr[j] = s.saddr[j]; }
        t.nexthdr = s.nexthdr;
        t.dport = t.sport = 0;
        return ct_l4<true>(t, s.h, CT_INGRESS, seen) >= 0;
    }
}

// the ICMP twin ct_create makes beside a new entry (conntrack.h ct_create4 / ct_create6)
template <bool V6, class T>
__device__ __forceinline__ T twin_of(const T &t2)
{
    T tw = t2;
    tw.nexthdr = V6 ? 58u : 1u;
    tw.sport = 0; tw.dport = 0;
    tw.flags = t2.flags | TUPLE_F_RELATED;
    return tw;
}

// What the earlier members' events say of keys ks[0..2] (the packet's tuple, its reverse,
// the reverse's ICMP twin): st[q] = 0 absent, 1 present, 2 untouched in this window
// (the table as the window started decides).  The latest confirmed event on a key
// counts: a delete leaves it absent, a create present iff the member's budget covered
// it (a failed create leaves it absent, as it was).  *used: a state came from a budget.
template <bool V6, class T>
__device__ __forceinline__ bool changed_state(const DpParams &p, const BatchDev &b, const GroupScratch &g,
                                              const Changed<T> &cg, const uint32_t (&ks)[3][T::KW],
                                              const uint8_t *budget, uint32_t (&st)[3], bool &used)
{
    if (cg.spill) {                                               // the run's table: the latest event per key
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            st[q] = 2;
            const uint32_t e = cg.find(key_hash<typename T::Spec>(ks[q]));
            if (e == ~0u) continue;
            const uint32_t m = e & 0x3FFFFFFFu, kind = e >> 30;
            T te;
            EpDev ep;
            uint32_t src;
            if (!intent_tuple<V6>(p, b, g, m, te, ep, src)) return false;
            te.reverse();
            if (kind == 2) te = twin_of<V6>(te);
            uint32_t km[T::KW];
            te.key(km);
            bool eq = true;
#pragma unroll
            for (int w = 0; w < T::KW; ++w) eq &= km[w] == ks[q][w];
            if (!eq) return false;                                // (a hash collision: unsure)
            if (kind) used = true;
            st[q] = kind ? (budget[m] >= kind ? 1u : 0u) : 0u;
        }
        return true;
    }
    uint32_t hit[3], all = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        st[q] = 2;
        const uint64_t hk = key_hash<typename T::Spec>(ks[q]);
        hit[q] = 0;
#pragma unroll
        for (int j = 0; j < Changed<T>::N; ++j) hit[q] |= (j < cg.n && cg.h[j] == hk) ? 1u << j : 0u;
        all |= hit[q];
    }
    while (all) {                                                 // latest first
        const int j = 31 - __clz(all);
        all &= ~(1u << j);
        uint32_t e = 0;
#pragma unroll
        for (int q = 0; q < Changed<T>::N; ++q) e = q == j ? cg.ev[q] : e;
        const uint32_t m = e & 0x3FFFFFFFu, kind = e >> 30;
        T te;
        EpDev ep;
        uint32_t src;
        if (!intent_tuple<V6>(p, b, g, m, te, ep, src)) continue;
        te.reverse();
        if (kind == 2) te = twin_of<V6>(te);
        uint32_t km[T::KW];
        te.key(km);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (st[q] != 2 || !((hit[q] >> j) & 1u)) continue;
            bool eq = true;
#pragma unroll
            for (int w = 0; w < T::KW; ++w) eq &= km[w] == ks[q][w];
            if (!eq) continue;                                    // (a hash collision)
            if (kind) used = true;
            st[q] = kind ? (budget[m] >= kind ? 1u : 0u) : 0u;
        }
    }
    return true;
}

// one packet's creates (bits 0-1), delete (bit 2) and unsure flag (bit 6, bit 7 the
// reason: too many changed keys in its run for Changed to hold)
template <bool V6, class T>
__device__ __forceinline__ uint32_t ct_intent(const DpParams &p, const BatchDev &b, const GroupScratch &g, uint32_t i,
                                              Changed<T> &cg, const uint8_t *budget, bool &used)
{
    T t;
    EpDev ep;
    uint32_t src;
    const bool any = intent_tuple<V6>(p, b, g, i, t, ep, src);
    if (!any) return 0;
    if (cg.overflow()) return 64u | 128u;
    const HashTable &ct = V6 ? ep.ct6 : ep.ct4;
    T t2 = t;
    t2.reverse();
    const T tw = twin_of<V6>(t2);
    uint32_t ks[3][T::KW], st[3];
    t.key(ks[0]);
    t2.key(ks[1]);
    tw.key(ks[2]);
    if (!changed_state<V6>(p, b, g, cg, ks, budget, st, used)) return 64u | 128u;
    auto present = [&](int q) { return st[q] == 2 ? dev_find<typename T::Spec>(ct, ks[q], nullptr) >= 0 : st[q] == 1; };
    if (present(0)) return 0;                                     // CT_REPLY / CT_RELATED
    const bool est = present(1);
    const bool deny = policy_ingress_denies(ep.policy, p.flags, src, t2.dport, t2.nexthdr);
    if (est) {
        if (!deny) return 0;
        cg.add(t2, i, 0);
        return 4u;                                                // ct_delete
    }
    if (deny) return 0;
    const uint32_t A = present(2) ? 1u : 2u;                      // (an existing twin is overwritten)
    cg.add(t2, i, 1);
    if (A == 2) cg.add(tw, i, 2);
    return A;
}

// ib bits besides A / D / map: 32 the intent read an earlier member's budget, 64 unsure,
// 128 (with 64) the reason: too many changed keys in the run
constexpr uint32_t IB_USED = 32u, IB_UNSURE = 64u;

// Pass 0 of a window replays every packet from a.lo; a later pass (a.pass) only the
// runs with a member whose intent read a budget (or that was unsure) in the previous
// one: the other intents cannot change (singletons never read one).
template <bool V6>
__global__ void __launch_bounds__(BLOCK) k_ct_intent(DpParams p, BatchDev b, GroupScratch g, Admit a)
{
    using T = typename std::conditional<V6, Tuple6, Tuple4>::type;
    const int q = V6 ? Q_NETDEV6 : Q_NETDEV;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    Changed<T> cg;
    auto one = [&](uint32_t x) {
        bool used = false;
        const uint32_t v = ct_intent<V6>(p, b, g, x, cg, a.budget, used);
        const uint32_t e = g.srec[2 * x + 1].z & 0xFFFFu;        // the destination endpoint
        uint32_t mi = e < p.n_eps ? (V6 ? a.ep_mi6 : a.ep_mi4)[e] : ADMIT_NO_MAP;
        if (mi >= a.nmaps) {                                      // (no conntrack stage: no intent)
            if (v) atomicOr(a.hi + 3, ADMIT_ERR_MAP);
            mi = 0;
        }
        const uint32_t nv = v | (used ? IB_USED : 0u), old = a.ib[x];
        a.ib[x] = (uint8_t)nv;
        if (v & 7u) a.mi[x] = (uint16_t)mi;
        if (v & IB_UNSURE) atomicMin(a.hi, x);
        if ((nv ^ old) & ~IB_USED) atomicMin(a.hi + 1, x);
        if (used) atomicMin(a.hi + 2, x);
    };
    uint32_t multi = 0;                                           // scheduled runs: classes >= 1
#pragma unroll
    for (int c = 1; c < NCLASS; ++c) multi += g.cursor[qcls(q, c)];
    for (uint32_t j = tid; j < multi; j += stride) {
        const uint32_t off = g.work[j];
        if (off >= 2u * g.lim) { group_err(g, GERR_INDEX); continue; }
        const uint32_t cnt = g.order[off];
        if (!run_ok(g, off, cnt)) continue;
        if (a.pass) {
            bool redo = false;
            for (uint32_t k = 0; k < cnt && !redo; ++k) {
                const uint32_t x = g.order[off + 1 + k];
                redo = pkt_ok(g, x) && x >= a.lo && (a.ib[x] & (IB_USED | IB_UNSURE));
            }
            if (!redo) continue;
        }
        cg.reset();
        if (cnt > 2 && a.evt) {                                   // (a spill table, should the run need one)
            cg.tab = a.evt + 2 * 4 * (size_t)off;
            cg.cap = 4 * (cnt + 1);
            cg.stamp = a.stamp;
        }
#pragma unroll 1
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint32_t x = g.order[off + 1 + k];
            if (pkt_ok(g, x) && x >= a.lo) one(x);                // (below: run by an earlier window)
        }
    }
    if (a.pass) return;
    const uint32_t singles = g.cursor[SINGLE_WORD0 + q];
    for (uint32_t j = tid; j < singles; j += stride) {
        const uint32_t x = g.single[j];
        cg.reset();
        if (pkt_ok(g, x) && x >= a.lo) one(x);
    }
}

__global__ void k_admit_init(Admit a, uint32_t n)
{
    if (threadIdx.x < 5 && blockIdx.x == 0) a.hi[threadIdx.x] = threadIdx.x < 3 ? n : 0u;
}

// test hook: a packet with one create whose map index is past the launch's maps
__global__ void k_admit_inject(Admit a)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        a.ib[a.inject] = (uint8_t)((a.ib[a.inject] & ~7u) | 1u);
        a.mi[a.inject] = (uint16_t)a.nmaps;
    }
}

// The reflected walk's two scans as one, over the monoid of (sum, prefix minimum) pairs:
// (s1, m1) then (s2, m2) = (s1 + s2, min(m1, s1 + m2)); a packet contributes (D - A, D - A)
// to its map's walk.  Every map's walk at once: the packets with creates or deletes,
// keyed map << 32 | packet and sorted (cv_sort.hip), are one sequence whose maps are
// segments; a head flag restarts the pair at a segment's first element, (f1, p1) then
// (f2, p2) = (f1 | f2, f2 ? p2 : p1 then p2).  Three kernels: tile aggregates, their
// exclusive scan, and a pass that rescans each tile and writes the budgets directly.
struct SumMin {
    int32_t s, m;
};
constexpr int32_t SM_INF = 1 << 30;                               // (|sums| <= 2^25: no overflow)

__device__ __forceinline__ SumMin sm_comb(SumMin l, SumMin r) { return {l.s + r.s, min(l.m, l.s + r.m)}; }

__device__ __forceinline__ SumMin sm_shfl_up(SumMin v, int d)
{
    return {__shfl_up(v.s, d, 64), __shfl_up(v.m, d, 64)};
}

// exclusive scan of one SumMin per thread over a block of 1024 (16 waves); *total: the
// block's aggregate
__device__ __forceinline__ SumMin block_excl_summin(SumMin v, SumMin *lds, SumMin *total)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    SumMin incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const SumMin t = sm_shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl = sm_comb(t, incl);
    }
    if (lane == 63) lds[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        SumMin acc{0, SM_INF};
        for (uint32_t w = 0; w < nw; ++w) { const SumMin t = lds[w]; lds[w] = acc; acc = sm_comb(acc, t); }
        lds[16] = acc;
    }
    __syncthreads();
    SumMin ex = sm_shfl_up(incl, 1);
    if (!lane) ex = SumMin{0, SM_INF};
    const SumMin r = sm_comb(lds[wv], ex);
    if (total) *total = lds[16];
    __syncthreads();
    return r;
}

// the segmented form: (f, s, m), f = a segment starts inside
struct SegSM {
    int32_t f, s, m;
};
__device__ __forceinline__ SegSM seg_comb(SegSM l, SegSM r)
{
    return r.f ? r : SegSM{l.f, l.s + r.s, min(l.m, l.s + r.m)};
}
__device__ __forceinline__ SegSM seg_shfl_up(SegSM v, int d)
{
    return {__shfl_up(v.f, d, 64), __shfl_up(v.s, d, 64), __shfl_up(v.m, d, 64)};
}
constexpr SegSM SEG_ID{0, 0, SM_INF};

__device__ __forceinline__ SegSM block_excl_seg(SegSM v, SegSM *lds, SegSM *total)
{
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    SegSM incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const SegSM t = seg_shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl = seg_comb(t, incl);
    }
    if (lane == 63) lds[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        SegSM acc = SEG_ID;
        for (uint32_t w = 0; w < nw; ++w) { const SegSM t = lds[w]; lds[w] = acc; acc = seg_comb(acc, t); }
        lds[16] = acc;
    }
    __syncthreads();
    SegSM ex = seg_shfl_up(incl, 1);
    if (!lane) ex = SEG_ID;
    const SegSM r = seg_comb(lds[wv], ex);
    if (total) *total = lds[16];
    __syncthreads();
    return r;
}

// the walks' elements: map << 24 | packet for the packets from lo with creates or
// deletes, appended in any order (the sort orders them); hi[4] counts them.  A block
// takes ADM_KPT packets per thread, contiguous, and allocates once per block (one
// returning atomic per lane-wave on one word serialised at the device's atomic rate:
// 2.9 ms per 2^24 packets)
constexpr uint32_t ADM_KPT = 16;
__global__ void __launch_bounds__(BLOCK) k_adm_keys(Admit a, uint32_t n)
{
    __shared__ uint32_t wsum[17], base_s;
    const uint32_t per = BLOCK * ADM_KPT;
    for (uint32_t b0 = a.lo + blockIdx.x * per; b0 < n; b0 += gridDim.x * per) {   // (block-uniform)
        const uint32_t j0 = b0 + threadIdx.x * ADM_KPT;
        uint32_t mine = 0;
#pragma unroll
        for (uint32_t u = 0; u < ADM_KPT; ++u) {
            const uint32_t j = j0 + u;
            if (j < n && (a.ib[j] & 7u)) ++mine;
        }
        uint32_t total;
        uint32_t at = block_excl_scan(mine, wsum, total);
        if (threadIdx.x == 0) base_s = total ? atomicAdd(a.hi + 4, total) : 0u;
        __syncthreads();
        at += base_s;
#pragma unroll
        for (uint32_t u = 0; u < ADM_KPT; ++u) {
            const uint32_t j = j0 + u;
            if (j >= n || !(a.ib[j] & 7u)) continue;
            const uint32_t mi = a.mi[j];
            unsigned long long k = (unsigned long long)mi << 24 | j;   // (j < MAX_CHUNK = 2^24)
            if (mi >= a.nmaps) {                                  // (a corrupt or stale map index)
                atomicOr(a.hi + 3, ADMIT_ERR_IB);
                k = (unsigned long long)(a.nmaps) << 24 | j;      // (sorted past every map, never applied)
            }
            a.keys[at++] = k;
        }
        __syncthreads();
    }
}

constexpr uint32_t KEY_NONE = 0xFFFFu;                            // (no element)
__device__ __forceinline__ uint32_t key_map(unsigned long long k) { return (uint32_t)(k >> 24) & 0xFFFFu; }

// element q of the sorted sequence (L of them): its map, packet, walk step and head flag
__device__ __forceinline__ SegSM adm_elem(const Admit &a, uint32_t L, uint32_t q, uint32_t &map, uint32_t &pkt)
{
    map = KEY_NONE;
    pkt = 0;
    if (q >= L) return SEG_ID;
    const unsigned long long k = a.keys_sorted[q];
    map = key_map(k);
    pkt = (uint32_t)k & 0xFFFFFFu;
    if (map >= a.nmaps) {                                         // (a corrupt element: never applied)
        map = KEY_NONE;
        return SEG_ID;
    }
    const uint32_t v = a.ib[pkt];
    const int32_t d = (int32_t)((v >> 2) & 1u) - (int32_t)(v & 3u);
    const int32_t f = q == 0 || key_map(a.keys_sorted[q - 1]) != map;
    return SegSM{f, d, d};
}

__global__ void __launch_bounds__(1024) k_adm_tiles(Admit a, uint32_t L)
{
    __shared__ SegSM lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    SegSM t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t m, x;
        t = seg_comb(t, adm_elem(a, L, j + k, m, x));
    }
    SegSM tot;
    block_excl_seg(t, lds, &tot);
    if (threadIdx.x == 0) reinterpret_cast<SegSM *>(a.tsum)[blockIdx.x] = tot;
}

// one block: the tile aggregates -> exclusive prefixes, in place
__global__ void __launch_bounds__(1024) k_adm_top(Admit a, uint32_t tiles)
{
    __shared__ SegSM lds[17];
    SegSM *agg = reinterpret_cast<SegSM *>(a.tsum);
    SegSM v[4], t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = threadIdx.x * 4 + k;
        v[k] = q < tiles ? agg[q] : SEG_ID;
        t = seg_comb(t, v[k]);
    }
    SegSM e = block_excl_seg(t, lds, nullptr);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = threadIdx.x * 4 + k;
        if (q < tiles) agg[q] = e;
        e = seg_comb(e, v[k]);
    }
}

// the budgets: the room before packet j is r0 + S - min(0, r0 + M) with (S, M) the
// walk's (sum, prefix minimum) over the earlier elements of j's map (r0 before lo)
__global__ void __launch_bounds__(1024) k_adm_apply(Admit a, uint32_t L)
{
    __shared__ SegSM lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    uint32_t map[4], pkt[4];
    SegSM e[4], t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        e[k] = adm_elem(a, L, j + k, map[k], pkt[k]);
        t = seg_comb(t, e[k]);
    }
    SegSM P = seg_comb(reinterpret_cast<const SegSM *>(a.tsum)[blockIdx.x], block_excl_seg(t, lds, nullptr));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (map[k] == KEY_NONE) continue;
        if (e[k].f) P = SEG_ID;                                   // (the map's first element)
        const uint32_t A = a.ib[pkt[k]] & 3u;
        if (A) {
            const unsigned long long live = __hip_atomic_load(a.live[map[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long r0 = live < a.cap[map[k]] ? (long long)(a.cap[map[k]] - live) : 0;
            const long long lowest = r0 + P.m < 0 ? r0 + P.m : 0;
            const long long r = r0 + P.s - lowest;
            a.budget[pkt[k]] = (uint8_t)(r < (long long)A ? r : (long long)A);
        }
        P = seg_comb(P, SegSM{0, e[k].s, e[k].m});
    }
}

// every packet from lo: budget 0 until the walks give it one
__global__ void __launch_bounds__(BLOCK) k_adm_zero(Admit a, uint32_t n)
{
    for (uint32_t j = a.lo + blockIdx.x * BLOCK + threadIdx.x; j < n; j += gridDim.x * BLOCK) a.budget[j] = 0;
}

int launch_admission(const DpParams &p, const BatchDev &b, const GroupScratch &g0, const Admit &a, hipStream_t s)
{
    GroupScratch g = g0;
    g.lim = b.n;
    if (!b.n || a.lo >= b.n) return 0;
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    if (a.nmaps >= KEY_NONE) return -EINVAL;
    hipLaunchKernelGGL(k_admit_init, dim3(1), dim3(64), 0, s, a, b.n);
    hipLaunchKernelGGL(k_ct_intent<false>, grid, blk, 0, s, p, b, g, a);
    GroupScratch g6 = g;
    g6.single = g.single6;
    g6.work = g.work6;
    hipLaunchKernelGGL(k_ct_intent<true>, grid, blk, 0, s, p, b, g6, a);
    if (a.inject >= a.lo && a.inject < b.n) hipLaunchKernelGGL(k_admit_inject, dim3(1), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_adm_keys, grid, blk, 0, s, a, b.n);
    return launch_status(__func__);
}

// the walks over the K elements k_adm_keys listed (a.hi[4], read by the host): sort,
// tile aggregates, their scan, the budgets
int launch_admission_walks(const BatchDev &b, const Admit &a, uint32_t K, hipStream_t s)
{
    if (!b.n || a.lo >= b.n) return 0;
    const dim3 grid(grid_for(b.n)), blk(BLOCK);
    const uint32_t tiles = (K + SCAN_TILE - 1) / SCAN_TILE;
    if (tiles > 4096 || K > b.n - a.lo) return -EINVAL;
    hipLaunchKernelGGL(k_adm_zero, grid, blk, 0, s, a, b.n);
    if (!K) return launch_status(__func__);
    int bits = 24;                                                // packet bits, then the map index's
    while ((1u << (bits - 24)) < a.nmaps) ++bits;
    size_t bytes = a.sort_bytes;
    if (int r = sort_keys64(a.sort_tmp, &bytes, a.keys, a.keys_sorted, K, bits, s)) return r;
    hipLaunchKernelGGL(k_adm_tiles, dim3(tiles), dim3(1024), 0, s, a, K);
    hipLaunchKernelGGL(k_adm_top, dim3(1), dim3(1024), 0, s, a, tiles);
    hipLaunchKernelGGL(k_adm_apply, dim3(tiles), dim3(1024), 0, s, a, K);
    return launch_status(__func__);
}

// ------------------------------------------------------------------ egress admission
// The budgets of an egress window (cv_ctx.cpp lxc_admitted) from what a pass recorded
// (EgAdm in cv_egress.hip): per packet the creates it tried, t (a failing one included:
// it ends the packet), and its deletes, d.  A packet's creates come before its delete
// (its service, conntrack and delivery stages; the delete is the delivery's), so per CT
// map its element of the (sum, prefix minimum) walk is (d - t, t ? -t : d), and the room
// before it is R = r0 + S - min(0, r0 + M).  The pass was the sequential run exactly when
// every packet got min(t, R) creates -- min(t, b) with b the budget it ran with: then the
// walk subtracted what the pass consumed, and a create failed exactly where the map was
// full.  The next pass's budgets are min(7, R) (generous: a packet that now creates more
// than it did finds room if the map has it).
__device__ __forceinline__ SumMin eadm_elem(uint32_t v, uint32_t m)
{
    const int32_t A = (int32_t)(v & 7u), D = (int32_t)((v >> 3) & 1u);
    if (((v >> 4) & 1u) != m || (!A && !D)) return SumMin{0, SM_INF};
    return SumMin{D - A, A ? -A : D};
}

__device__ __forceinline__ uint32_t eadm_v4(const EAdmit &a, uint32_t j)
{
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (j + k < a.n) w |= (uint32_t)a.intent[j + k] << (8 * k);
    return w;
}

__global__ void __launch_bounds__(1024) k_eadm_tiles(EAdmit a, uint32_t tiles)
{
    __shared__ SumMin lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    const uint32_t w = eadm_v4(a, j);
    SumMin *agg = reinterpret_cast<SumMin *>(a.tsum);
    for (uint32_t m = 0; m < 2; ++m) {
        SumMin t{0, SM_INF};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (j + k < a.n) t = sm_comb(t, eadm_elem(w >> (8 * k) & 0xFFu, m));
        SumMin tot;
        block_excl_summin(t, lds, &tot);
        if (threadIdx.x == 0) agg[m * tiles + blockIdx.x] = tot;
    }
}

__global__ void __launch_bounds__(1024) k_eadm_top(EAdmit a, uint32_t tiles)
{
    __shared__ SumMin lds[17];
    SumMin *agg = reinterpret_cast<SumMin *>(a.tsum);
    for (uint32_t m = 0; m < 2; ++m) {
        SumMin v[4], t{0, SM_INF};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = threadIdx.x * 4 + k;
            v[k] = q < tiles ? agg[m * tiles + q] : SumMin{0, SM_INF};
            t = sm_comb(t, v[k]);
        }
        SumMin e = block_excl_summin(t, lds, nullptr);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = threadIdx.x * 4 + k;
            if (q < tiles) agg[m * tiles + q] = e;
            e = sm_comb(e, v[k]);
        }
    }
}

__global__ void __launch_bounds__(1024) k_eadm_apply(EAdmit a, uint32_t tiles)
{
    __shared__ SumMin lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    const uint32_t w = eadm_v4(a, j);
    const SumMin *agg = reinterpret_cast<const SumMin *>(a.tsum);
    uint32_t out = 0;
    bool bad = false;
    for (uint32_t m = 0; m < 2; ++m) {
        SumMin t{0, SM_INF};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (j + k < a.n) t = sm_comb(t, eadm_elem(w >> (8 * k) & 0xFFu, m));
        SumMin P = sm_comb(agg[m * tiles + blockIdx.x], block_excl_summin(t, lds, nullptr));
        const unsigned long long live = *a.live0[m];
        const long long r0 = live < a.cap[m] ? (long long)(a.cap[m] - live) : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t v = w >> (8 * k) & 0xFFu, t = v & 7u;
            if (((v >> 4) & 1u) == m && j + k < a.n) {
                const long long lowest = r0 + P.m < 0 ? r0 + P.m : 0;
                const long long R = r0 + P.s - lowest;
                const uint32_t b = a.used[j + k];
                bad |= (uint32_t)(R < (long long)t ? R : (long long)t) != (t < b ? t : b);
                out |= (uint32_t)(R < 7 ? R : 7) << (8 * k);
            }
            P = sm_comb(P, eadm_elem(v, m));
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (j + k < a.n) a.next[j + k] = (uint8_t)(out >> (8 * k));
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(a.flag, 1u);
}

int launch_egress_admission(const EAdmit &a, hipStream_t s)
{
    if (!a.n) return 0;
    const uint32_t tiles = (a.n + SCAN_TILE - 1) / SCAN_TILE;
    if (tiles > 4096) return -EINVAL;
    (void)hipMemsetAsync(a.flag, 0, 4, s);
    hipLaunchKernelGGL(k_eadm_tiles, dim3(tiles), dim3(1024), 0, s, a, tiles);
    hipLaunchKernelGGL(k_eadm_top, dim3(1), dim3(1024), 0, s, a, tiles);
    hipLaunchKernelGGL(k_eadm_apply, dim3(tiles), dim3(1024), 0, s, a, tiles);
    return launch_status(__func__);
}

// ------------------------------------------------------------------ egress admission, many CT maps
// (cv_ctx.cpp lxc_admitted_maps; EAdmitM in cv_dp.hpp).  A packet's slot-0 element is its
// source program's creates and delete in its source endpoint's map, its slot-1 element
// its local delivery's in the destination's map; per map the elements in packet order
// (slot 0 before slot 1 of one packet) are a walk of (d - t, t ? -t : d) steps, as one CT
// map's packets are in the one-budget form above.
__device__ __forceinline__ uint32_t eam_map(const EAdmitM &a, uint32_t j, uint32_t slot)
{
    const uint32_t f = (a.intent[j] >> 4) & 1u;
    const uint32_t e = slot ? a.dst_ep[j] : a.src_ep ? a.src_ep[j] : a.ep0;
    return e < a.n_eps ? (f ? a.ep_mi6 : a.ep_mi4)[e] : ADMIT_NO_MAP;
}

// A slot is an element when it ran in the pass -- the source program of a packet past the
// front (intent bit 32), a delivery that reached its destination (dst_ep set) -- with or
// without creates: then the next pass gives it the room at its place in its map's walk
// (a packet that created nothing here may try to in the next pass, once an earlier create
// it hit fails; a stale budget would let it succeed where the map is full, one more pass
// per such packet of a flow)
__device__ __forceinline__ bool eam_has(const EAdmitM &a, uint32_t j, uint32_t slot)
{
    return slot ? (a.dst_ep[j] != 0xFFFFu || (a.intent2[j] & 15u)) : (a.intent[j] & 47u) != 0;
}

// first pass: 7 creates per element, none in a source map that is full
__global__ void __launch_bounds__(BLOCK) k_eam_first(EAdmitM a)
{
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < a.n; j += gridDim.x * BLOCK) {
        const uint32_t e = a.src_ep ? a.src_ep[j] : a.ep0;
        uint32_t mi4 = e < a.n_eps ? a.ep_mi4[e] : ADMIT_NO_MAP, mi6 = e < a.n_eps ? a.ep_mi6[e] : ADMIT_NO_MAP;
        const bool room4 = mi4 < a.nmaps && a.live0[mi4] < a.cap[mi4];
        const bool room6 = mi6 < a.nmaps && a.live0[mi6] < a.cap[mi6];
        // (the family is not known before the front: room in either map gives 7, the
        // check corrects a guess that was too generous)
        a.next[j] = room4 || room6 ? 7u : 0u;
        a.next2[j] = 7u;
    }
}

// the elements from their intents: map << 25 | packet << 1 | slot, appended in any order
// (block-aggregated allocation, as k_adm_keys)
__global__ void __launch_bounds__(BLOCK) k_eam_keys(EAdmitM a)
{
    __shared__ uint32_t wsum[17], base_s;
    const uint32_t per = BLOCK * ADM_KPT;
    for (uint32_t b0 = blockIdx.x * per; b0 < a.n; b0 += gridDim.x * per) {   // (block-uniform)
        const uint32_t j0 = b0 + threadIdx.x * ADM_KPT;
        uint32_t mine = 0;
#pragma unroll
        for (uint32_t u = 0; u < ADM_KPT; ++u) {
            const uint32_t j = j0 + u;
            if (j < a.n) mine += (eam_has(a, j, 0) ? 1u : 0u) + (eam_has(a, j, 1) ? 1u : 0u);
        }
        uint32_t total;
        uint32_t at = block_excl_scan(mine, wsum, total);
        if (threadIdx.x == 0) base_s = total ? atomicAdd(a.cnt, total) : 0u;
        __syncthreads();
        at += base_s;
#pragma unroll
        for (uint32_t u = 0; u < ADM_KPT; ++u) {
            const uint32_t j = j0 + u;
            if (j >= a.n) continue;
            for (uint32_t sl = 0; sl < 2; ++sl) {
                if (!eam_has(a, j, sl)) continue;
                uint32_t mi = eam_map(a, j, sl);
                if (mi >= a.nmaps) {                              // (a create in a map not in the list)
                    atomicOr(a.cnt + 2, 1u);
                    mi = a.nmaps;                                 // (sorted past every map, never applied)
                }
                a.keys[at++] = (unsigned long long)mi << 25 | (unsigned long long)j << 1 | sl;
            }
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint32_t eam_key_map(unsigned long long k) { return (uint32_t)(k >> 25) & 0xFFFFu; }

__device__ __forceinline__ SegSM eam_elem(const EAdmitM &a, uint32_t L, uint32_t q, uint32_t &map, uint32_t &pkt,
                                          uint32_t &slot)
{
    map = KEY_NONE;
    pkt = slot = 0;
    if (q >= L) return SEG_ID;
    const unsigned long long k = a.keys_sorted[q];
    map = eam_key_map(k);
    pkt = (uint32_t)(k >> 1) & 0xFFFFFFu;
    slot = (uint32_t)k & 1u;
    if (map >= a.nmaps || pkt >= a.n) {
        map = KEY_NONE;
        return SEG_ID;
    }
    const uint32_t v = (slot ? a.intent2 : a.intent)[pkt];
    const int32_t A = (int32_t)(v & 7u), D = (int32_t)((v >> 3) & 1u);
    const int32_t f = q == 0 || eam_key_map(a.keys_sorted[q - 1]) != map;
    return SegSM{f, D - A, A ? -A : D};
}

__global__ void __launch_bounds__(1024) k_eam_tiles(EAdmitM a, uint32_t L)
{
    __shared__ SegSM lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    SegSM t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t m, x, sl;
        t = seg_comb(t, eam_elem(a, L, j + k, m, x, sl));
    }
    SegSM tot;
    block_excl_seg(t, lds, &tot);
    if (threadIdx.x == 0) reinterpret_cast<SegSM *>(a.tsum)[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) k_eam_top(EAdmitM a, uint32_t tiles)
{
    __shared__ SegSM lds[17];
    SegSM *agg = reinterpret_cast<SegSM *>(a.tsum);
    SegSM v[4], t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = threadIdx.x * 4 + k;
        v[k] = q < tiles ? agg[q] : SEG_ID;
        t = seg_comb(t, v[k]);
    }
    SegSM e = block_excl_seg(t, lds, nullptr);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t q = threadIdx.x * 4 + k;
        if (q < tiles) agg[q] = e;
        e = seg_comb(e, v[k]);
    }
}

// per element the room before it, R = r0 + S - min(0, r0 + M): the pass was the sequential
// run iff min(t, b) = min(t, R) for every element (t its creates, b its budget); the next
// budget min(7, R)
__global__ void __launch_bounds__(1024) k_eam_apply(EAdmitM a, uint32_t L)
{
    __shared__ SegSM lds[17];
    const uint32_t j = blockIdx.x * SCAN_TILE + threadIdx.x * 4;
    uint32_t map[4], pkt[4], slot[4];
    SegSM e[4], t = SEG_ID;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        e[k] = eam_elem(a, L, j + k, map[k], pkt[k], slot[k]);
        t = seg_comb(t, e[k]);
    }
    SegSM P = seg_comb(reinterpret_cast<const SegSM *>(a.tsum)[blockIdx.x], block_excl_seg(t, lds, nullptr));
    uint32_t bad = 0, first = ~0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (map[k] == KEY_NONE) continue;
        if (e[k].f) P = SEG_ID;                                   // (the map's first element)
        const uint32_t v = (slot[k] ? a.intent2 : a.intent)[pkt[k]], A = v & 7u;
        const unsigned long long live = a.live0[map[k]];
        const long long r0 = live < a.cap[map[k]] ? (long long)(a.cap[map[k]] - live) : 0;
        const long long lowest = r0 + P.m < 0 ? r0 + P.m : 0;
        const long long R = r0 + P.s - lowest;
        const uint32_t b = (slot[k] ? a.used2 : a.used)[pkt[k]];
        if ((uint32_t)(R < (long long)A ? R : (long long)A) != (A < b ? A : b)) {
            ++bad;
            first = min(first, pkt[k]);
        }
        (slot[k] ? a.next2 : a.next)[pkt[k]] = (uint8_t)(R < 7 ? R : 7);
        P = seg_comb(P, SegSM{0, e[k].s, e[k].m});
    }
    for (int d = 32; d; d >>= 1) {                                // (per wave: the count, the first packet)
        bad += (uint32_t)__shfl_xor((int)bad, d, 64);
        first = min(first, (uint32_t)__shfl_xor((int)first, d, 64));
    }
    if (bad && (threadIdx.x & 63) == 0) {
        atomicAdd(a.cnt + 1, bad);
        atomicMin(a.cnt + 3, first);
    }
}

int launch_eam_first(const EAdmitM &a, hipStream_t s)
{
    if (!a.n) return 0;
    const uint32_t g = (a.n + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(k_eam_first, dim3(g < 2048 ? g : 2048), dim3(BLOCK), 0, s, a);
    return launch_status(__func__);
}

int launch_eam_keys(const EAdmitM &a, hipStream_t s)
{
    if (a.nmaps >= KEY_NONE || a.n > MAX_CHUNK) return -EINVAL;
    (void)hipMemsetAsync(a.cnt, 0, 12, s);
    (void)hipMemsetAsync(a.cnt + 3, 0xFF, 4, s);
    if (!a.n) return 0;
    const uint32_t per = BLOCK * ADM_KPT, g = (a.n + per - 1) / per;
    hipLaunchKernelGGL(k_eam_keys, dim3(g < 2048 ? g : 2048), dim3(BLOCK), 0, s, a);
    return launch_status(__func__);
}

// K elements (cnt[0], read by the host): sort, tile aggregates, their scan, the check and
// the next budgets (an element-less slot keeps the budget it ran with: the caller copies
// used -> next first)
int launch_eam_walks(const EAdmitM &a, uint32_t K, hipStream_t s)
{
    const uint32_t tiles = (K + SCAN_TILE - 1) / SCAN_TILE;
    if (tiles > 4096 || K > 2 * a.n) return -EINVAL;
    if (!K) return 0;
    int bits = 25;                                                // packet and slot bits, then the map index's
    while ((1u << (bits - 25)) <= a.nmaps) ++bits;                // (nmaps itself: the corrupt elements)
    size_t bytes = a.sort_bytes;
    if (int r = sort_keys64(a.sort_tmp, &bytes, a.keys, a.keys_sorted, K, bits, s)) return r;
    hipLaunchKernelGGL(k_eam_tiles, dim3(tiles), dim3(1024), 0, s, a, K);
    hipLaunchKernelGGL(k_eam_top, dim3(1), dim3(1024), 0, s, a, tiles);
    hipLaunchKernelGGL(k_eam_apply, dim3(tiles), dim3(1024), 0, s, a, K);
    return launch_status(__func__);
}

// A pass undone (Snap, cv_dp.hpp): every logged slot back as it was -- its bucket words,
// side slot and tag byte (a CAS on the tag word, which other slots of the bucket share).
// Each slot is logged once per pass (its spare-word bit).
__device__ __forceinline__ bool snap_used(const Snap &sn, uint32_t e)
{
    return e % SNAP_PER < sn.cnt[e / SNAP_PER];
}

__device__ __forceinline__ uint32_t *snap_bucket(const uint4 *d)
{
    const uint4 h0 = d[0];
    return reinterpret_cast<uint32_t *>((uintptr_t)((unsigned long long)h0.y << 32 | h0.x));
}

__global__ void __launch_bounds__(BLOCK) k_snap_restore(Snap sn)
{
    for (uint32_t e = blockIdx.x * BLOCK + threadIdx.x; e < sn.n * SNAP_PER; e += gridDim.x * BLOCK) {
        if (!snap_used(sn, e)) continue;
        const uint4 *d = sn.log + (size_t)e * SNAP_U4;
        uint32_t *bw = snap_bucket(d);
        const uint32_t meta = d[0].z, parts = d[0].w, s = meta & 0xFFu, tag = (meta >> 8) & 0xFFu,
                       ks = (meta >> 16) & 0xFFu;
        if (ks > 20) continue;                                    // (not a CT slot record)
        const uint32_t *w = reinterpret_cast<const uint32_t *>(d);
        if (parts & 2u) {                                         // (SNAP_COLD: the side slot)
            const uint4 q = d[8];
            uint32_t *cold = reinterpret_cast<uint32_t *>((uintptr_t)((unsigned long long)q.y << 32 | q.x));
            for (uint32_t j = 0; j < 8; ++j) cold[j] = w[24 + j];
        }
        if (!(parts & 1u)) continue;                              // (SNAP_HOT: bucket words and tag)
        uint32_t *kw = bw + 2 + s * ks;                           // (KEY0 = 2 for both CT specs)
        for (uint32_t j = 0; j < ks; ++j) kw[j] = w[4 + j];
        uint32_t *tw = bw + (s >> 2);
        const uint32_t sh = 8 * (s & 3);
        uint32_t c = __hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            const uint32_t nw = (c & ~(0xFFu << sh)) | (tag << sh);
            if (__hip_atomic_compare_exchange_strong(tw, &c, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT))
                break;
        }
    }
}

// after every pass: the logged slots' bits in their buckets' spare words back to 0
__global__ void __launch_bounds__(BLOCK) k_snap_clear(Snap sn)
{
    for (uint32_t e = blockIdx.x * BLOCK + threadIdx.x; e < sn.n * SNAP_PER; e += gridDim.x * BLOCK) {
        if (!snap_used(sn, e)) continue;
        const uint4 *d = sn.log + (size_t)e * SNAP_U4;
        const uint32_t meta = d[0].z, s = meta & 0xFFu, parts = d[0].w;
        atomicAnd(snap_bucket(d) + (meta >> 24), ~(((parts & 1u) ? 1u << s : 0u) | ((parts & 2u) ? 1u << (8 + s) : 0u)));
    }
}

int launch_snap_restore(const Snap &sn, hipStream_t s)
{
    const uint32_t g = (sn.n * SNAP_PER / BLOCK) + 1;
    hipLaunchKernelGGL(k_snap_restore, dim3(g < 4096 ? g : 4096), dim3(BLOCK), 0, s, sn);
    return launch_status(__func__);
}

int launch_snap_clear(const Snap &sn, hipStream_t s)
{
    const uint32_t g = (sn.n * SNAP_PER / BLOCK) + 1;
    hipLaunchKernelGGL(k_snap_clear, dim3(g < 4096 ? g : 4096), dim3(BLOCK), 0, s, sn);
    return launch_status(__func__);
}

__global__ void __launch_bounds__(BLOCK) k_scatter_u64(unsigned long long *const *ptrs, const unsigned long long *in,
                                                       uint32_t n)
{
    for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < n; k += gridDim.x * BLOCK)
        __hip_atomic_store(ptrs[k], in[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int launch_scatter_u64(unsigned long long *const *ptrs, const unsigned long long *in, uint32_t n, hipStream_t s)
{
    if (!n) return 0;
    const uint32_t g = (n + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(k_scatter_u64, dim3(g < 1024 ? g : 1024), dim3(BLOCK), 0, s, ptrs, in, n);
    return launch_status(__func__);
}

// the agent's staged table writes (cv_ctx.cpp PatchQueue): a block per run of words
__global__ void __launch_bounds__(BLOCK) k_patch(const PatchRec *recs, uint32_t n, const uint32_t *words)
{
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const PatchRec pr = recs[r];
        uint32_t *dst = reinterpret_cast<uint32_t *>(pr.dst);
        for (uint32_t w = threadIdx.x; w < pr.words; w += BLOCK) dst[w] = words[pr.src + w];
    }
}

int launch_patches(const PatchRec *recs, uint32_t n, const uint32_t *words, hipStream_t s)
{
    if (!n) return 0;
    hipLaunchKernelGGL(k_patch, dim3(n < 4096 ? n : 4096), dim3(BLOCK), 0, s, recs, n, words);
    return launch_status(__func__);
}

int launch_ct_op(const HashTable &t, int v6, int op, uint64_t flags, uint32_t *io_dev, hipStream_t s)
{
    hipLaunchKernelGGL(k_ct_op, dim3(1), dim3(64), 0, s, t, v6, op, flags, io_dev);
    return launch_status(__func__);
}

int launch_ct_scan(const HashTable &t, int v6, uint64_t nb, uint64_t *out_slots, uint32_t *out_keys, uint32_t *out_vals,
                   uint32_t *count, uint32_t max, hipStream_t s)
{
    const uint64_t slots = nb * (v6 ? Ct6Spec::SPB : Ct4Spec::SPB);
    uint64_t g = (slots + BLOCK - 1) / BLOCK;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_ct_scan, dim3((uint32_t)g), dim3(BLOCK), 0, s, t, v6, slots, out_slots, out_keys, out_vals,
                       count, max);
    return launch_status(__func__);
}

}  // namespace cv
