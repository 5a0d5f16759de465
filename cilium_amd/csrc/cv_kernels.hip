// cv_kernels.hip — gfx950 kernels of the batch verdict engine, ingress side.
//
// One lane = one packet.  Each kernel restates a path of the reference's BPF
// programs (Taeung/cilium v1.1.90) over a batch of frame records in HBM:
//   k_xdp_prefilter    bpf/bpf_xdp.c:88-184                      (config 1)
//   k_policy_ingress   bpf/bpf_netdev.c:128-153,357-398 +
//                      bpf/lib/policy.h:217-329                   (config 2)
//   k_netdev_front     bpf/bpf_netdev.c:357-524, bpf/lib/l3.h:247-276
//   k_ct_stage         bpf/bpf_lxc.c:865-1038, bpf/lib/conntrack.h (config 3)
// The egress path (config 5) is in cv_egress.hip; the shared device functions
// (map probes, policy, conntrack, metrics, grouping) in cv_dev.hpp.  No MFMA: this
// is integer gather work, HBM/L2 bound.
#include "cv_dev.hpp"

namespace cv {

// ================================================================== config 1
// A wave's record load and probes: wave-cooperative 1-KiB record loads through LDS
// when the wave's 64 records are all in the batch (64-B stride), quad probes
// (cv_hash.hpp) for the tables; the loops are wave-uniform so every lane reaches
// every probe (lanes past the end with live = false).
__device__ __forceinline__ void rec_load_wave(Rec &r, const DpParams &p, const BatchDev &b, uint32_t i0, uint32_t i,
                                              bool live, uint4 *st)
{
    if (p.recmode == 2 && b.stride == 64 && i0 + 64 <= b.n) rec_load_wave64(r, b, i0, 4, st);
    else if (!live) { r.len = 0; for (int j = 0; j < 16; ++j) r.w[j] = 0; }
    else rec_load(r, b, i, 4);
}

// The config-2 verdict words leave as streaming (nontemporal) stores: the output
// lines are never read back by the launch, so they do not take L2 / Infinity Cache
// room from the table lines (config 2: 0.886 -> 0.870 ms, profiles/r01y/ab_nt*).
template <class T>
__device__ __forceinline__ void st_out(T *q, T v)
{
#ifdef CV_NO_NT_OUT            // A/B only
    *q = v;
#else
    __builtin_nontemporal_store(v, q);
#endif
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
// lookup is done.
#ifndef CV_PPT
#define CV_PPT 4
#endif
constexpr int PPT = CV_PPT;

#ifndef CV_NO_QUAD
// Quad-probe form: the table probes are quad_find (cv_hash.hpp), so every lane of
// the wave reaches each probe; lanes without a lookup (past the batch end, non-IPv4,
// short or invalid headers) take part with want = false.  (Holding the results in
// registers until after the last probe, so the probes' vmcnt waits skip the output
// stores, measured 3 % slower.)
#ifdef CV_PI_WPE               // A/B only
#define CV_PI_OCC __attribute__((amdgpu_waves_per_eu(CV_PI_WPE, 8)))
#else
#define CV_PI_OCC
#endif
__global__ void __launch_bounds__(BLOCK) CV_PI_OCC k_policy_ingress(DpParams p, int ep, BatchDev b, OutDev o)
{
    __shared__ unsigned long long drops[256 * 2];                 // ingress drops {count, bytes} by reason
#ifdef CV_POL_PAIR
    __shared__ uint4 stage[BLOCK / 64][512];
#else
    __shared__ uint4 stage[BLOCK / 64][256];
#endif
    for (int j = threadIdx.x; j < 256 * 2; j += BLOCK) drops[j] = 0;
    __syncthreads();
    const HashTable pol = p.eps[ep].policy;
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
        if (p.recmode == 2 && b.stride == 64 && i0 + 64 <= b.n) rec_load_wave64(r, b, i0, 3, st);
        else if (!live) { r.len = 0; for (int j = 0; j < 16; ++j) r.w[j] = 0; }
        else if (p.recmode == 1) rec_load_plain(r, b, i, 3);
        else rec_load(r, b, i, 3);
        Acct a{0, 0};
        bool skip_proxy = false;
        uint32_t identity = 0;
        if (live && (p.flags & F_FROM_HOST)) identity = identity_from_mark(b.mark ? b.mark[i] : 0u, skip_proxy);
        const uint32_t eth = r.len >= 14 ? rec_raw16c<12>(r) : 0u;
        const bool v4 = live && eth == 0x0008u && r.len >= 34;
        const bool want_ipc = v4 && identity < HEALTH_ID && !(p.ablate & AB_NO_IPCACHE);   // bpf_netdev.c:375-398
        const uint32_t lab = ipcache4_q(p, rec_raw32c<26>(r), want_ipc, a, st);
        if (want_ipc && lab && lab != CLUSTER_ID && lab != HOST_ID) identity = lab;
        int32_t ret = eth != 0x0008u ? DROP_UNKNOWN_L3 : r.len < 34 ? DROP_INVALID : 0;
        uint32_t dport = 0, proto = 0;
        if (v4) ret = l4_key_new_flow(r, dport, proto);
        const bool want_pol = v4 && ret == 0 && !(p.ablate & AB_NO_POLICY);
        const int v = policy_ingress_q(pol, p.flags | (p.ablate << 16), r.len, identity, dport, proto, a, &hits[k],
                                       want_pol, st);
        uint16_t proxy = 0;
        if (v4 && ret == 0) {
            const int vv = (p.ablate & AB_NO_POLICY) ? (int)(identity & 1) : v;
            if (vv < 0) ret = DROP_POLICY;
            else if (skip_proxy && vv > 0) ret = 0;
            else { ret = vv; proxy = vv > 0 ? (uint16_t)vv : 0; }
        }
        if (!live) continue;
        const bool dropped = ret < 0 && ret != E_TRUNC;
        if (dropped && !(p.ablate & AB_NO_METRICS)) {             // send_drop_notify -> cilium_metrics
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
#else
__global__ void __launch_bounds__(BLOCK) k_policy_ingress(DpParams p, int ep, BatchDev b, OutDev o)
{
    __shared__ LdsMetrics lm;
    __shared__ uint4 stage[BLOCK / 64][256];
    MetT<false> m;
    met_init(m, lm);
    const HashTable pol = p.eps[ep].policy;
    Hit hits[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        hits[k] = Hit{nullptr, 0};
        const uint32_t i = blockIdx.x * (PPT * BLOCK) + k * BLOCK + threadIdx.x;
        const uint32_t i0 = i - (threadIdx.x & 63);
        Rec r;
        if (p.recmode == 2 && b.stride == 64 && i0 + 64 <= b.n) rec_load_wave64(r, b, i0, 3, stage[threadIdx.x >> 6]);
        else if (i >= b.n) continue;
        else if (p.recmode == 1) rec_load_plain(r, b, i, 3);
        else rec_load(r, b, i, 3);
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
        const bool dropped = ret < 0 && ret != E_TRUNC;
        if (dropped && !(p.ablate & AB_NO_METRICS)) m.drop(ret, r.len, METRIC_INGRESS);
        if (o.ret) o.ret[i] = ret;
        if (o.reason) o.reason[i] = dropped ? ret : 0;
        if (o.identity) o.identity[i] = identity;
        if (o.proxy) o.proxy[i] = proxy;
        if (o.ct) o.ct[i] = CT_NONE;
        store_out(o, i, a);
    }
#pragma unroll
    for (int k = 0; k < PPT; ++k) hit_flush(hits[k]);
    met_flush(m, p.metrics);
}
#endif

// ================================================================== config 3
// stage 1: XDP prefilter + from_netdev/handle_ipv4 up to the tail call into the
// endpoint's policy program; packets reaching it join their address-pair group.
#ifdef CV_NF_WPE               // A/B only
#define CV_NF_OCC __attribute__((amdgpu_waves_per_eu(CV_NF_WPE, 8)))
#else
#define CV_NF_OCC
#endif
template <bool EV>
__global__ void __launch_bounds__(BLOCK) CV_NF_OCC k_netdev_front(DpParams p, BatchDev b, OutDev o, GroupScratch g,
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
        uint8_t xv = XDP_PASS;
        int32_t ret = TC_ACT_OK, reason = 0;
        uint32_t ident = 0;
        bool staged = false;
        if (with_prefilter) xv = xdp_verdict_q(p, r, a, live, st);
        const bool pass = live && xv == XDP_PASS;
        bool skip_proxy = false;
        uint32_t identity = 0;
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
            }
        }
        const bool want_lxc = v4 && h == TC_ACT_OK && p.lxc4.buckets;
        if (want_lxc) a.nl++;                                     // lookup_ip4_endpoint
        uint32_t iv = 0;
        uint32_t daddr = rec_raw32c<30>(r);
        const int64_t lxc_slot = quad_find<LxcV4Spec>(p.lxc4, &daddr, want_lxc, st, &iv);
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
                        g.secctx[i] = secctx;
                        g.meta[i] = (e - 1) | (skip_proxy ? 1u << 16 : 0u) | ((iv >> 17) & 1u) << 17;
                        if (EV) g.ifx[i] = (uint32_t)lxc_slot;    // -> cb[CB_IFINDEX], MACs (stage 2)
                    }
                }
            }
            if (!staged) {
                if (h == E_TRUNC) ret = h;
                else if (is_err(h)) {                             // tail_handle_ipv4: send_drop_notify_error
                    m.drop(h, r.len, METRIC_INGRESS);
                    m.pkt = b.base + i;
                    m.hash = b.hash ? b.hash[i] : 0u;
                    notify_drop(p, m, h, r.len, 0, 0, 0, 0, 0);
                    reason = h;
                    ret = TC_ACT_SHOT;
                }
                else ret = h;
            }
        }
        if (staged) {                                             // group by (CT map, address pair)
            const EpDev &ep = p.eps[g.meta[i] & 0xFFFFu];
            group_push(g, group_node(g, pair_hash4(rec_raw32c<26>(r), daddr, (uint64_t)ep.ct_id << 17)), i, Q_NETDEV);
        }
        if (!live) continue;
        if (M::EV && o.frames) frame_copy(b.frames + (size_t)i * b.stride, o.frames + (size_t)i * b.stride, b.stride);
        if (!staged) {
            g.gslot[i] = NONE;
            if (o.ret) o.ret[i] = ret;
            if (o.reason) o.reason[i] = reason;
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
    met_flush(m, p.metrics);
}

template <class M>
__device__ __forceinline__ void stage2_one(const DpParams &p, const BatchDev &b, const OutDev &o,
                                           const GroupScratch &g, uint32_t i, uint32_t now, M &m)
{
    Rec r;
    rec_load(r, b, i, 3);
    const uint32_t meta = g.meta[i];
    const EpDev &ep = p.eps[meta & 0xFFFFu];
    Acct a{o.nl ? o.nl[i] : 0u, o.nu ? o.nu[i] : 0u, m.pc};
    uint8_t ct = CT_NONE;
    uint16_t proxy = 0;
    int32_t reason = 0;
    Skb4 s = skb4_from(r);
    int64_t lslot = -1;                                          // the destination's cilium_lxc slot
    if constexpr (M::EV) {
        m.pkt = b.base + i;
        m.hash = b.hash ? b.hash[i] : 0u;
        lslot = (int32_t)g.ifx[i];
    }
    RevNatOut rn{false, false, 0, 0};
    const int ret = handle_policy4(p, ep, s, g.secctx[i], (meta >> 16) & 1u,
                                   ifindex_of(m, p.lxc4, lslot, ((meta >> 17) & 1u) << 17), now, ct, proxy, reason,
                                   a, m, &rn);
    if (M::EV && o.frames && (ret == TC_ACT_OK || ret == TC_ACT_REDIRECT) && !proxy) {
        // the forwarded frame: ipv4_local_delivery's ipv4_l3 (bpf_netdev handle_ipv4), then
        // the policy program's reverse NAT
        const uint8_t *in = b.frames + (size_t)i * b.stride;
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

#ifdef CV_CT_WPE               // A/B only: 121 VGPRs give 4 waves/SIMD already; 5 is slower
#define CV_CT_OCC __attribute__((amdgpu_waves_per_eu(CV_CT_WPE, 8)))
#else
#define CV_CT_OCC
#endif

// stage 2: conntrack + policy, each address-pair group by one lane in packet order
template <bool EV>
__global__ void __launch_bounds__(BLOCK) CV_CT_OCC k_ct_stage(DpParams p, BatchDev b, OutDev o, GroupScratch g, uint32_t now)
{
    __shared__ LdsMetrics lm;
    __shared__ LdsPolicy pc;
    MetT<EV> m;
    pol_cache_init(pc);
    met_init(m, lm);
    m.pc = &pc;
#if CV_RUNS_MODE == 0
    for_each_group(g, Q_NETDEV, [&](uint32_t, uint32_t head) {
        group_in_order(g, head, 0, [&](uint32_t x) { stage2_one(p, b, o, g, x, now, m); });
    });
#else
    for_each_run<CV_RUNS_MODE != 2>(g, Q_NETDEV, false, [&](uint32_t x) { stage2_one(p, b, o, g, x, now, m); });
#endif
    met_flush(m, p.metrics);                                      // (ends with a barrier)
    pol_cache_flush(pc);
}

// ------------------------------------------------------------------ size-sorted runs
// k_group_flatten: every queued group of q becomes a run {size, members ascending}
// in `order` (one block-aggregated allocation per 256 groups); the queue word is
// replaced by the run's offset; per-class counts.  Block-uniform loop (the scans use
// every lane).
__global__ void __launch_bounds__(BLOCK) k_group_flatten(GroupScratch g, int q)
{
    __shared__ uint32_t hist[NCLASS], wsum[BLOCK / 64], bbase;
    if (threadIdx.x < NCLASS) hist[threadIdx.x] = 0;
    uint32_t n[QSPLIT];
    const uint32_t total = queue_sizes(g, q, n);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t base = blockIdx.x * BLOCK; base < total; base += gridDim.x * BLOCK) {
        const uint32_t j = base + threadIdx.x;
        const bool act = j < total;
        uint32_t *ent = nullptr, cnt = 0, x = NONE, head = NONE;
        uint32_t m[GMAX];
        if (act) {
            ent = queue_entry(g, q, n, j);
            head = (uint32_t)g.table[2 * *ent + 1];
            for (x = head; x != NONE && cnt < GMAX; x = g.next[x]) {   // insertion into registers
                int pos = 0;
#pragma unroll
                for (int t = 0; t < GMAX; ++t) pos += (t < (int)cnt && m[t] < x) ? 1 : 0;
#pragma unroll
                for (int t = GMAX - 1; t >= 0; --t) {
                    const uint32_t left = t > 0 ? m[t - 1] : 0u;
                    m[t] = (t < pos) ? m[t] : (t == pos ? x : left);
                }
                ++cnt;
            }
            for (uint32_t y = x; y != NONE; y = g.next[y]) ++cnt;
        }
        const uint32_t need = act ? cnt + 1 : 0;
        uint32_t incl = need;                                     // wave inclusive scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += t;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int w = 0; w < BLOCK / 64; ++w) { const uint32_t t = wsum[w]; wsum[w] = acc; acc += t; }
            bbase = acc ? atomicAdd(&g.cursor[RUN_CURSOR], acc) : 0;
        }
        __syncthreads();
        if (act) {
            const uint32_t off = bbase + wsum[wv] + incl - need;
            uint32_t *o = g.order + off;
            o[0] = cnt;
            if (cnt <= GMAX) {
#pragma unroll
                for (int t = 0; t < GMAX; ++t)
                    if (t < (int)cnt) o[1 + t] = m[t];
            } else {                                              // large group: copy, shell sort
                uint32_t k = 1;
                for (uint32_t y = head; y != NONE; y = g.next[y]) o[k++] = y;
                ++o;
                for (uint32_t gap = cnt / 2; gap > 0; gap = gap == 2 ? 1 : gap * 5 / 11) {
                    for (uint32_t i = gap; i < cnt; ++i) {
                        const uint32_t v = o[i];
                        uint32_t t = i;
                        for (; t >= gap && o[t - gap] > v; t -= gap) o[t] = o[t - gap];
                        o[t] = v;
                    }
                }
            }
            *ent = off;
            atomicAdd(&hist[size_class(cnt)], 1u);
        }
        uint32_t big = cnt;                                       // the largest group (diagnostics)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) big = max(big, (uint32_t)__shfl_xor(big, d, 64));
        if (lane == 0 && big > 8) atomicMax(&g.cursor[GMAX_WORD0 + q], big);
        __syncthreads();                                          // wsum / bbase reuse
    }
    __syncthreads();
    if (threadIdx.x < NCLASS && hist[threadIdx.x]) atomicAdd(&g.cursor[qcls(q, threadIdx.x)], hist[threadIdx.x]);
}

// k_group_schedule: `work` lists the runs class by class, largest class first
constexpr int SCHED_PER_THREAD = 4;
__global__ void __launch_bounds__(BLOCK) k_group_schedule(GroupScratch g, int q, bool largest_first)
{
    __shared__ uint32_t cbase[NCLASS], lcnt[NCLASS], lbase[NCLASS];
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < NCLASS; ++k) {
            const int c = largest_first ? NCLASS - 1 - k : k;
            cbase[c] = acc;
            acc += g.cursor[qcls(q, c)];
        }
    }
    uint32_t n[QSPLIT];
    const uint32_t total = queue_sizes(g, q, n);
    constexpr uint32_t SPAN = BLOCK * SCHED_PER_THREAD;
    for (uint32_t base = blockIdx.x * SPAN; base < total; base += gridDim.x * SPAN) {
        if (threadIdx.x < NCLASS) lcnt[threadIdx.x] = 0;
        __syncthreads();
        uint32_t off[SCHED_PER_THREAD], cls[SCHED_PER_THREAD], rank[SCHED_PER_THREAD];
#pragma unroll
        for (int u = 0; u < SCHED_PER_THREAD; ++u) {
            const uint32_t j = base + u * BLOCK + threadIdx.x;
            if (j < total) {
                off[u] = *queue_entry(g, q, n, j);
                cls[u] = size_class(g.order[off[u]]);
                rank[u] = atomicAdd(&lcnt[cls[u]], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x < NCLASS && lcnt[threadIdx.x])
            lbase[threadIdx.x] = atomicAdd(&g.cursor[qcls(q, threadIdx.x) + 1], lcnt[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < SCHED_PER_THREAD; ++u) {
            const uint32_t j = base + u * BLOCK + threadIdx.x;
            if (j < total) g.work[cbase[cls[u]] + lbase[cls[u]] + rank[u]] = off[u];
        }
        __syncthreads();
    }
}

void launch_group_runs(const GroupScratch &g, int q, int grid, int sched, hipStream_t s)
{
    hipLaunchKernelGGL(k_group_flatten, dim3(grid), dim3(BLOCK), 0, s, g, q);
    if (sched) hipLaunchKernelGGL(k_group_schedule, dim3(grid), dim3(BLOCK), 0, s, g, q, sched == 1);
}

// ------------------------------------------------------------------ CT map API
// Single-element BPF_MAP_{LOOKUP,UPDATE,DELETE}_ELEM on a device-resident CT table
// (the agent side of pkg/maps/ctmap: GC deletes, dumps, restores).
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
            ct_load(t, s, e);
            for (int k = 0; k < 16; ++k) val[k] = e.w[k];
        }
    } else if (op == 1) {
        if (s >= 0 && flags == 1) rc = -EEXIST;
        else if (s < 0 && flags == 2) rc = -ENOENT;
        else {
            bool created;
            s = dev_upsert<S>(t, key, &created);
            if (s < 0) rc = -E2BIG;
            else {
                CtE e;
                for (int k = 0; k < 16; ++k) e.w[k] = val[k];
                ct_store(t, s, e);
            }
        }
    } else {
        if (s < 0) rc = -ENOENT;
        else dev_kill<S>(t, s);
    }
    *rcp = (uint32_t)rc;
}

__global__ void k_ct_op(HashTable t, int v6, int op, uint64_t flags, uint32_t *io)
{
    if (threadIdx.x || blockIdx.x) return;
    if (v6) ct_op<Ct6Spec>(t, op, flags, io);
    else ct_op<Ct4Spec>(t, op, flags, io);
}

// compact every live entry (tag >= 3) into key/value arrays
template <class S>
__device__ void ct_scan(HashTable t, uint64_t nslots, uint32_t *keys, uint32_t *vals, uint32_t *count, uint32_t max)
{
    for (uint64_t x = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; x < nslots; x += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t b = x / S::SPB;
        const int sl = (int)(x % S::SPB);
        const uint32_t *bw = t.buckets + b * S::BW;
        const uint32_t tag = (bw[sl >> 2] >> (8 * (sl & 3))) & 0xFFu;
        if (tag < 3) continue;
        const uint32_t at = atomicAdd(count, 1u);
        if (at >= max) continue;
        for (int j = 0; j < S::KW; ++j) keys[(size_t)at * S::KW + j] = bw[S::KEY0 + sl * S::KW + j];
        const uint32_t *v = reinterpret_cast<const uint32_t *>(t.vals + x * t.vstride);
        for (int j = 0; j < 16; ++j) vals[(size_t)at * 16 + j] = v[j];
    }
}

__global__ void k_ct_scan(HashTable t, int v6, uint64_t nslots, uint32_t *keys, uint32_t *vals, uint32_t *count,
                          uint32_t max)
{
    if (v6) ct_scan<Ct6Spec>(t, nslots, keys, vals, count, max);
    else ct_scan<Ct4Spec>(t, nslots, keys, vals, count, max);
}

// ctmap.GC with GCFilterByTime (pkg/maps/ctmap/ctmap.go:325-432): one pass over the
// table, a lane per bucket: read the 8 tag bytes, then the lifetime word of every
// live slot, and mark the expired ones dead (the bucket's tag word rewritten once;
// the pass runs stream-ordered between batches, so it is the only writer).
template <class S>
__device__ void ct_gc(HashTable t, uint64_t nb, uint32_t time, uint32_t *deleted)
{
    uint32_t mine = 0;
    for (uint64_t b = blockIdx.x * (uint64_t)BLOCK + threadIdx.x; b < nb; b += (uint64_t)gridDim.x * BLOCK) {
        uint32_t *bw = t.buckets + b * S::BW;
        const uint2 tg = *reinterpret_cast<const uint2 *>(bw);
        uint64_t tags = (uint64_t)tg.x | ((uint64_t)tg.y << 32), out = tags;
#pragma unroll
        for (int sl = 0; sl < S::SPB; ++sl) {
            const uint32_t tag = (uint32_t)(tags >> (8 * sl)) & 0xFFu;
            if (tag < 3) continue;
            const uint32_t life = *reinterpret_cast<const uint32_t *>(t.vals + (b * S::SPB + sl) * t.vstride + 32);
            if (life < time) {
                out = (out & ~(0xFFull << (8 * sl))) | ((uint64_t)TAG_DEAD << (8 * sl));
                ++mine;
            }
        }
        if (out != tags) *reinterpret_cast<uint2 *>(bw) = make_uint2((uint32_t)out, (uint32_t)(out >> 32));
    }
    const unsigned long long tot = wave_sum(mine);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(deleted, (uint32_t)tot);
}

__global__ void __launch_bounds__(BLOCK) k_ct_gc(HashTable t, int v6, uint64_t nb, uint32_t time, uint32_t *deleted)
{
    if (v6) ct_gc<Ct6Spec>(t, nb, time, deleted);
    else ct_gc<Ct4Spec>(t, nb, time, deleted);
}

int launch_ct_gc(const HashTable &t, int v6, uint64_t nb, uint32_t time, uint32_t *deleted, hipStream_t s)
{
    uint64_t g = (nb + BLOCK - 1) / BLOCK;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_ct_gc, dim3((uint32_t)(g ? g : 1)), dim3(BLOCK), 0, s, t, v6, nb, time, deleted);
    return hipGetLastError() == hipSuccess ? 0 : -5;
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
    const bool ev = o.frames || p.notify || p.trace;              // the instance with the optional outputs
    if (ev) hipLaunchKernelGGL(k_netdev_front<true>, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, with_prefilter);
    else hipLaunchKernelGGL(k_netdev_front<false>, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, with_prefilter);
    if (hipGetLastError() != hipSuccess) return -5;
    if (CV_RUNS_MODE) launch_group_runs(g, Q_NETDEV, grid_for(b.n), runs_sched(CV_RUNS_MODE), s);
    if (ev) hipLaunchKernelGGL(k_ct_stage<true>, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, now);
    else hipLaunchKernelGGL(k_ct_stage<false>, dim3(grid_for(b.n)), dim3(BLOCK), 0, s, p, b, o, g, now);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ct_op(const HashTable &t, int v6, int op, uint64_t flags, uint32_t *io_dev, hipStream_t s)
{
    hipLaunchKernelGGL(k_ct_op, dim3(1), dim3(64), 0, s, t, v6, op, flags, io_dev);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ct_scan(const HashTable &t, int v6, uint64_t nb, uint32_t *out_keys, uint32_t *out_vals, uint32_t *count,
                   uint32_t max, hipStream_t s)
{
    const uint64_t slots = nb * (v6 ? Ct6Spec::SPB : Ct4Spec::SPB);
    uint64_t g = (slots + BLOCK - 1) / BLOCK;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_ct_scan, dim3((uint32_t)g), dim3(BLOCK), 0, s, t, v6, slots, out_keys, out_vals, count, max);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace cv
