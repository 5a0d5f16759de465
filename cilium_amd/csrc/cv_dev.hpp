// cv_dev.hpp — device-side building blocks shared by the gfx950 kernels: frame
// records in registers, the per-packet "skb" view after rewrites, map probes,
// policy, conntrack (v4 and v6), reverse NAT, cilium_metrics aggregation and the
// address-pair grouping that gives a batch sequential (one-CPU) semantics.
//
// Every function restates a function of the reference (Taeung/cilium v1.1.90) and
// cites it; the CPU restatement in oracle/cv_oracle.c follows the same lines.
#pragma once
#include <errno.h>
#include <hip/hip_runtime.h>

#include "cv_dp.hpp"

namespace cv {

constexpr int BLOCK = 256;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t COMMIT4 = 0xFFFFFFFEu;     // g.gslot marks of a deferred CT create (k_ct_commit)
constexpr uint32_t COMMIT6 = 0xFFFFFFFDu;
constexpr uint32_t COMMIT_PROXY = 2u;         // COMMIT4/6 - 2: the packet went to the proxy (no forward metric)

// ------------------------------------------------------------------ records
// The first 4*NW bytes of a frame record live in NW VGPRs (loaded with 16-B
// non-temporal loads, so streamed records do not evict tables from L2 / MALL);
// bytes at runtime offsets outside the common layout come from HBM.
template <int NW>
struct RecT {
    uint32_t w[NW];
    const uint8_t *base;
    uint32_t len, stride;
};
using Rec = RecT<16>;    // IPv4: Ethernet + IPv4 + L4 in 64 B
using Rec6 = RecT<32>;   // IPv6: Ethernet + IPv6 + L4 in 128 B

template <int NW>
__device__ __forceinline__ void rec_load(RecT<NW> &r, const BatchDev &b, uint32_t i, int nvec)
{
    r.base = b.frames + (size_t)i * b.stride;
    r.len = b.len[i];
    r.stride = b.stride;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *q = reinterpret_cast<const u32x4 *>(r.base);
#pragma unroll
    for (int k = 0; k < NW / 4; ++k) {
        if (k < nvec) {
            u32x4 v = __builtin_nontemporal_load(q + k);
            r.w[4 * k] = v.x; r.w[4 * k + 1] = v.y; r.w[4 * k + 2] = v.z; r.w[4 * k + 3] = v.w;
        } else {
            r.w[4 * k] = r.w[4 * k + 1] = r.w[4 * k + 2] = r.w[4 * k + 3] = 0;
        }
    }
}

// Wave-cooperative load of the 64 consecutive 64-B records of a wave (i0 = the
// wave's first packet): four fully coalesced 1-KiB loads per wave into LDS (`st`,
// 4 KiB per wave), then every lane takes its own record's first nvec 16-B words.
// Uniform per wave; the caller falls back to per-lane loads for partial waves.
__device__ __forceinline__ void rec_load_wave64(Rec &r, const BatchDev &b, uint32_t i0, int nvec, uint4 *st)
{
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(b.frames + (size_t)i0 * 64);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const u32x4 v = __builtin_nontemporal_load(src + c * 64 + lane);
        const int chunk = c * 64 + lane;                          // record chunk/4, part chunk%4
        st[(chunk & 3) * 64 + (chunk >> 2)] = make_uint4(v.x, v.y, v.z, v.w);   // part-major: conflict-free reads
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t i = i0 + lane;
    r.base = b.frames + (size_t)i * 64;
    r.len = b.len[i];
    r.stride = 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k < nvec) {
            const uint4 v = st[k * 64 + lane];
            r.w[4 * k] = v.x; r.w[4 * k + 1] = v.y; r.w[4 * k + 2] = v.z; r.w[4 * k + 3] = v.w;
        } else {
            r.w[4 * k] = r.w[4 * k + 1] = r.w[4 * k + 2] = r.w[4 * k + 3] = 0;
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// The same for records of any register width (NW / 4 16-B parts, stride 4 * NW): the
// wave's 64 consecutive records in NW / 4 fully coalesced 1-KiB loads through LDS
// (`st`: 16 * NW uint4 per wave).  All 64 lanes, wave-uniform, i0 + 64 <= b.n.
template <int NW>
__device__ __forceinline__ void rec_load_coop(RecT<NW> &r, const BatchDev &b, uint32_t i0, uint4 *st)
{
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr int P = NW / 4;
    const int lane = threadIdx.x & 63;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(b.frames + (size_t)i0 * (4 * NW));
#pragma unroll
    for (int c = 0; c < P; ++c) {
        const u32x4 v = __builtin_nontemporal_load(src + c * 64 + lane);
        const int chunk = c * 64 + lane;                          // record chunk / P, part chunk % P
        st[(chunk % P) * 64 + chunk / P] = make_uint4(v.x, v.y, v.z, v.w);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t i = i0 + lane;
    r.base = b.frames + (size_t)i * (4 * NW);
    r.len = b.len[i];
    r.stride = 4 * NW;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const uint4 v = st[k * 64 + lane];
        r.w[4 * k] = v.x; r.w[4 * k + 1] = v.y; r.w[4 * k + 2] = v.z; r.w[4 * k + 3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
}

// the first 16 words of a wider record (an IPv4 packet in a 128-B record)
template <int NW>
__device__ __forceinline__ Rec rec_head(const RecT<NW> &w)
{
    Rec r;
#pragma unroll
    for (int j = 0; j < 16; ++j) r.w[j] = w.w[j];
    r.base = w.base;
    r.len = w.len;
    r.stride = w.stride;
    return r;
}

template <int O, int NW>
__device__ __forceinline__ uint32_t rec_u8c(const RecT<NW> &r)
{
    static_assert(O >= 0 && O < 4 * NW, "register window");
    return (r.w[O >> 2] >> (8 * (O & 3))) & 0xFFu;
}

template <int O, int NW>
__device__ __forceinline__ uint32_t rec_raw16c(const RecT<NW> &r)   // raw LE load of 2 network-order bytes
{
    static_assert(O >= 0 && O + 2 <= 4 * NW, "register window");
    if constexpr ((O & 3) == 3) return rec_u8c<O>(r) | (rec_u8c<O + 1>(r) << 8);
    else return (r.w[O >> 2] >> (8 * (O & 3))) & 0xFFFFu;
}

template <int O, int NW>
__device__ __forceinline__ uint32_t rec_raw32c(const RecT<NW> &r)
{
    static_assert(O >= 0 && O + 4 <= 4 * NW, "register window");
    if constexpr ((O & 3) == 0) return r.w[O >> 2];
    else return (r.w[O >> 2] >> (8 * (O & 3))) | (r.w[(O >> 2) + 1] << (32 - 8 * (O & 3)));
}

// byte K of the L4 header at runtime offset `off`: registers when off == FAST
template <int FAST, int K, int NW>
__device__ __forceinline__ uint32_t l4_u8(const RecT<NW> &r, int off)
{
    if (off == FAST) return rec_u8c<FAST + K>(r);
    return r.base[off + K];
}

template <int FAST, int K, int NW>
__device__ __forceinline__ uint32_t l4_raw16(const RecT<NW> &r, int off)
{
    if (off == FAST) return rec_raw16c<FAST + K>(r);
    return r.base[off + K] | ((uint32_t)r.base[off + K + 1] << 8);
}

// skb_load_bytes / skb_store_bytes bound: 0 ok, 1 beyond skb->len (the helper
// fails), E_TRUNC inside len but beyond the record
template <int NW>
__device__ __forceinline__ int rec_chk(const RecT<NW> &r, int off, int n)
{
    if (off < 0 || (uint32_t)(off + n) > r.len) return 1;
    if ((uint32_t)(off + n) > r.stride) return E_TRUNC;
    return 0;
}

// rec_chk on a packet known only by its length and record stride
__device__ __forceinline__ int len_chk(uint32_t len, uint32_t stride, int off, int n)
{
    if (off < 0 || (uint32_t)(off + n) > len) return 1;
    if ((uint32_t)(off + n) > stride) return E_TRUNC;
    return 0;
}

// The L4 bytes the programs read, with the outcome of each load the reference
// does: [off,1) ICMP type, [off+12,2) TCP flags, [off,4) ports, [off,2) sport,
// [off+2,2) dport.  Rewrites (lb xlate, rev-NAT) update p0 / p2 in place, as the
// reference's skb_store_bytes would.
struct L4Hdr {
    int8_t c1, c14, c4, c2a, c2b;
    uint32_t type, tflags;
    uint32_t p0, p2;          // raw be16 of bytes 0-1 and 2-3
};

template <int FAST, int NW>
__device__ __forceinline__ L4Hdr l4_read(const RecT<NW> &r, int off)
{
    L4Hdr h;
    h.c1 = (int8_t)rec_chk(r, off, 1);
    h.c14 = (int8_t)rec_chk(r, off + 12, 2);
    h.c4 = (int8_t)rec_chk(r, off, 4);
    h.c2a = (int8_t)rec_chk(r, off, 2);
    h.c2b = (int8_t)rec_chk(r, off + 2, 2);
    h.type = h.c1 == 0 ? l4_u8<FAST, 0>(r, off) : 0u;
    h.tflags = h.c14 == 0 ? l4_u8<FAST, 13>(r, off) : 0u;
    h.p0 = h.c2a == 0 ? l4_raw16<FAST, 0>(r, off) : 0u;
    h.p2 = h.c2b == 0 ? l4_raw16<FAST, 2>(r, off) : 0u;
    return h;
}

__device__ __forceinline__ int chk_err(int c, int code) { return c == E_TRUNC ? E_TRUNC : code; }
__device__ __forceinline__ bool is_err(int x) { return x < 0 || x == TC_ACT_SHOT; }   // common.h:231

// ------------------------------------------------------------------ metrics
// cilium_metrics (metrics.h:43-58): drops go through a per-workgroup LDS table
// [256 reasons][2 dirs]{count, bytes}; forwards (reason 0, one per delivered packet)
// accumulate in the lane's registers and are wave-reduced once per kernel.
struct LdsMetrics {
    unsigned long long c[256 * 2 * 2];
};

struct Fwd {
    uint32_t c[2];
    unsigned long long b[2];
};

// Policy entry counters (the packets/bytes __policy_can_access adds to the hit entry)
// summed per workgroup: a direct-mapped LDS table keyed by the entry's delta-word
// address; a slot taken by another entry sends the update to global memory as
// before.  Flushed once per workgroup: hot entries (one L3 rule hit by most packets)
// see one global atomic per workgroup instead of one per packet.  Sums commute, so
// the folded counters equal the per-packet updates.
// The conntrack maps' live-entry counts (one word per map, added to by every create
// and delete of the launch) get slots of their own: in the shared table a policy
// entry holding their slot would send every create of the workgroup to that one
// global word, where returning and non-returning atomics alike serialise.
constexpr int PC_N = 256, PC_LIVE = 8;
struct LdsPolicy {
    unsigned long long key[PC_N];
    unsigned long long val[PC_N];
    unsigned long long lkey[PC_LIVE];
    unsigned long long lval[PC_LIVE];
};

__device__ __forceinline__ void pol_add(LdsPolicy *pc, unsigned long long *d, unsigned long long inc)
{
    if (pc) {
        const unsigned long long k = reinterpret_cast<uintptr_t>(d);
        const uint32_t i = (uint32_t)(mix64(k) >> 40) & (PC_N - 1);
        unsigned long long cur = pc->key[i];
        if (cur == 0) {
            unsigned long long exp = 0;
            __hip_atomic_compare_exchange_strong(&pc->key[i], &exp, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            cur = exp == 0 ? k : exp;
        }
        if (cur == k) {
            __hip_atomic_fetch_add(&pc->val[i], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
    }
    __hip_atomic_fetch_add(G(d), inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void live_add(LdsPolicy *pc, unsigned long long *d, unsigned long long inc)
{
    if (pc) {
        const unsigned long long k = reinterpret_cast<uintptr_t>(d);
#pragma unroll
        for (int i = 0; i < PC_LIVE; ++i) {
            unsigned long long cur = pc->lkey[i];
            if (cur == 0) {
                unsigned long long exp = 0;
                __hip_atomic_compare_exchange_strong(&pc->lkey[i], &exp, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                cur = exp == 0 ? k : exp;
            }
            if (cur == k) {
                __hip_atomic_fetch_add(&pc->lval[i], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return;
            }
        }
    }
    pol_add(pc, d, inc);
}

__device__ __forceinline__ void pol_cache_init(LdsPolicy &pc)
{
    for (int i = threadIdx.x; i < PC_N; i += blockDim.x) pc.key[i] = 0, pc.val[i] = 0;
    if (threadIdx.x < PC_LIVE) pc.lkey[threadIdx.x] = 0, pc.lval[threadIdx.x] = 0;
}

// after a __syncthreads that follows the workgroup's last pol_add
__device__ __forceinline__ void pol_cache_flush(const LdsPolicy &pc)
{
    for (int i = threadIdx.x; i < PC_N; i += blockDim.x)
        if (pc.key[i] && pc.val[i])
            __hip_atomic_fetch_add(G(reinterpret_cast<unsigned long long *>(pc.key[i])), pc.val[i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < PC_LIVE && pc.lkey[threadIdx.x] && pc.lval[threadIdx.x])
        __hip_atomic_fetch_add(G(reinterpret_cast<unsigned long long *>(pc.lkey[threadIdx.x])), pc.lval[threadIdx.x],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// EVENTS: the kernel instance that emits the optional outputs (drop / trace records,
// rewritten frames); the plain instance compiles them out (launchers pick one per call)
// SNAP: the egress admission instance with many CT maps (CT slots saved before their first
// write in a pass, Snap); the other instances compile the saving out
template <bool EVENTS, bool SNAP = false>
struct MetT {
    static constexpr bool EV = EVENTS, SN = SNAP;
    LdsMetrics *lm;
    Fwd f;
    LdsPolicy *pc;             // optional policy counter cache (conntrack stages)
    // the packet being processed, for drop notifications: batch index, skb hash, and
    // the sending endpoint program (egress: LXC_ID, SECLABEL)
    uint32_t pkt, hash, src_id, src_label;
    __device__ void drop(int32_t code, uint32_t len, int dir)          // send_drop_notify
    {
        const uint32_t r = (uint8_t)(-code);
        const int k = (r * 2 + (dir - 1)) * 2;
        atomicAdd(&lm->c[k], 1ull);
        atomicAdd(&lm->c[k + 1], (unsigned long long)len);
    }
    __device__ void fwd(uint32_t len, int dir)                         // update_metrics(.., REASON_FORWARDED)
    {
        f.c[dir - 1] += 1;
        f.b[dir - 1] += len;
    }
};

template <class M>
__device__ __forceinline__ void met_init(M &m, LdsMetrics &lm)
{
    for (int i = threadIdx.x; i < 256 * 4; i += blockDim.x) lm.c[i] = 0;
    m.lm = &lm;
    m.pc = nullptr;
    m.pkt = m.hash = m.src_id = m.src_label = 0;
    m.f.c[0] = m.f.c[1] = 0;
    m.f.b[0] = m.f.b[1] = 0;
    __syncthreads();
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <class M>
__device__ __forceinline__ void met_flush(M &m, unsigned long long *g)
{
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        const unsigned long long c = wave_sum(m.f.c[d]), b = wave_sum(m.f.b[d]);
        if ((threadIdx.x & 63) == 0 && c) {
            atomicAdd(&m.lm->c[(0 * 2 + d) * 2], c);
            atomicAdd(&m.lm->c[(0 * 2 + d) * 2 + 1], b);
        }
    }
    __syncthreads();
    if (!g) return;
    for (int i = threadIdx.x; i < 256 * 2; i += blockDim.x) {
        const int r = i >> 1, d = i & 1;
        const unsigned long long c = m.lm->c[i * 2];
        if (c) {
            atomicAdd(&g[(r * 4 + d + 1) * 2], c);
            atomicAdd(&g[(r * 4 + d + 1) * 2 + 1], m.lm->c[i * 2 + 1]);
        }
    }
}

// wave-aggregated append: one atomic per (wave, counter); lanes may target different
// counters; returns the lane's index or NONE
__device__ __forceinline__ uint32_t wave_append(uint32_t *ctr, bool pred)
{
    const int lane = (int)__lane_id();
    uint32_t res = NONE;
    unsigned long long todo = __ballot(pred);
    while (todo) {                                                // one round per distinct counter
        const int leader = __ffsll((long long)todo) - 1;
        const uintptr_t mine_p = reinterpret_cast<uintptr_t>(ctr);
        const uint32_t lo = __shfl((uint32_t)mine_p, leader, 64), hi = __shfl((uint32_t)(mine_p >> 32), leader, 64);
        uint32_t *lc = reinterpret_cast<uint32_t *>((uintptr_t)lo | ((uintptr_t)hi << 32));
        const bool mine = pred && ctr == lc;
        const unsigned long long m = __ballot(mine);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(lc, (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        if (mine) res = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        todo &= ~m;
    }
    return res;
}

// send_drop_notify -> __send_drop_notify (bpf/lib/drop.h:50-108): one cv_drop_notify
// record (10 words) per drop when a ring is attached; wave-aggregated slot claims
template <class M>
__device__ __forceinline__ void notify_drop(const DpParams &p, const M &m, int32_t code, uint32_t len,
                                            uint32_t source, uint32_t src, uint32_t dst, uint32_t dst_id,
                                            uint32_t ifindex)
{
    if constexpr (!M::EV) return;
    if (!p.notify) return;
    const uint32_t at = wave_append(p.notify_count, true);
    if (at >= p.notify_cap) return;                               // lost sample (ring full)
    const uint32_t srcdst = (src << 16) | (dst & 0xFFFFu);       // skb->cb[1]
    uint32_t *w = p.notify + (size_t)at * 10;
    const uint32_t sub = (uint32_t)(uint8_t)(code < 0 ? -code : code);
    *reinterpret_cast<uint4 *>(w) = make_uint4(1u | sub << 8 | (source & 0xFFFFu) << 16, m.hash, len,
                                               len < 128 ? len : 128u);
    *reinterpret_cast<uint4 *>(w + 4) = make_uint4(srcdst >> 16, srcdst & 0xFFFFu, dst_id, ifindex);
    *reinterpret_cast<uint2 *>(w + 8) = make_uint2(m.pkt, 0u);
}

// send_trace_notify (bpf/lib/trace.h:96-150): one cv_trace_notify record (10 words)
// per forwarding step when a ring is attached; FROM_* points hidden at
// MONITOR_AGGREGATION >= 1, steps without a CT report request at >= 3
enum : uint32_t { TRACE_TO_LXC = 0, TRACE_TO_PROXY = 1, TRACE_TO_HOST = 2, TRACE_TO_STACK = 3,
                  TRACE_FROM_LXC = 5, TRACE_FROM_PROXY = 6, TRACE_FROM_HOST = 7, TRACE_FROM_STACK = 8 };
template <class M>
__device__ __forceinline__ void notify_trace(const DpParams &p, const M &m, uint32_t obs, uint32_t len,
                                             uint32_t source, uint32_t src, uint32_t dst, uint32_t dst_id,
                                             uint32_t ifindex, uint32_t reason, bool monitor)
{
    if constexpr (!M::EV) return;
    if (!p.trace) return;
    if (p.trace_agg >= 1 && obs >= TRACE_FROM_LXC) return;
    if (p.trace_agg >= 3 && !monitor) return;
    const uint32_t at = wave_append(p.trace_count, true);
    if (at >= p.trace_cap) return;                                // lost sample (ring full)
    uint32_t *w = p.trace + (size_t)at * 10;
    *reinterpret_cast<uint4 *>(w) = make_uint4(4u | obs << 8 | (source & 0xFFFFu) << 16, m.hash, len,
                                               len < 128 ? len : 128u);
    *reinterpret_cast<uint4 *>(w + 4) = make_uint4(src, dst, (dst_id & 0xFFFFu) | (reason & 0xFFu) << 16, ifindex);
    *reinterpret_cast<uint2 *>(w + 8) = make_uint2(m.pkt, 0u);
}

// ------------------------------------------------------------------ lookups
struct Acct {
    uint32_t nl, nu;
    LdsPolicy *pc = nullptr;   // policy counter cache of the workgroup, if any
    uint32_t budget = ~0u;     // admission windows: creates of new CT entries that may still succeed
    uint32_t tried = 0;        // admission: creates of new entries tried (a failing one included)
    uint32_t killed = 0;       // admission: entries deleted
    const Snap *snap = nullptr;  // egress admission with many CT maps: slots saved before their first write
    uint32_t spkt = 0, scnt = 0;   // (the packet and its log entries so far)
    uint32_t ctu = 1;          // what a conntrack lookup / write adds to nl / nu (ACCT_CT_UNIT: the split)
};
// CV_F_ACCT_SPLIT: conntrack lookups and writes count ACCT_CT_UNIT in nl / nu, the other
// lookups and writes 1 -- one accounting pass gives the HBM-resident share of B(p)
constexpr uint32_t ACCT_CT_UNIT = 32;
__device__ __forceinline__ uint32_t ct_unit(const DpParams &p) { return (p.flags & F_ACCT_SPLIT) ? ACCT_CT_UNIT : 1u; }

// lookup_ip4_endpoint (eps.h:37-46): ival = lxc_id | HOST << 16 | (ifindex != 0) << 17
__device__ __forceinline__ bool lxc4_find(const DpParams &p, uint32_t daddr_raw, uint32_t &ival, Acct &a)
{
    if (!p.lxc4.buckets) return false;
    a.nl++;
    return dev_find<LxcV4Spec>(p.lxc4, &daddr_raw, &ival) >= 0;
}

// lookup_ip6_endpoint (eps.h:26-35)
__device__ __forceinline__ bool lxc6_find(const DpParams &p, const uint32_t *daddr, uint32_t &ival, Acct &a)
{
    if (!p.lxc6.buckets) return false;
    a.nl++;
    return dev_find<LxcV6Spec>(p.lxc6, daddr, &ival) >= 0;
}

// endpoint_info.ifindex of the matched cilium_lxc entry (the 4-B side value of its
// slot); without the side array, the inline nonzero bit
__device__ __forceinline__ uint32_t lxc_ifindex(const HashTable &t, int64_t slot, uint32_t ival)
{
    if (t.vals && slot >= 0) return *reinterpret_cast<const CV_G uint32_t *>(G(t.vals) + (size_t)slot * t.vstride);
    return (ival >> 17) & 1u;
}

// the ifindex a program hands on: the value itself where a record carries it (the
// event instances), else only whether it is nonzero (redirect vs TC_ACT_OK), which
// the inline bit answers without a dependent read of the side array
template <class M>
__device__ __forceinline__ uint32_t ifindex_of(const M &, const HashTable &t, int64_t slot, uint32_t ival)
{
    if constexpr (M::EV) return lxc_ifindex(t, slot, ival);
    else return (ival >> 17) & 1u;
}

// endpoint_info.mac / .node_mac of a matched cilium_lxc entry (words: bytes 0-3, 4-5)
__device__ __forceinline__ void lxc_macs(const HashTable &t, int64_t slot, uint32_t *mac, uint32_t *node_mac)
{
    const CV_G uint32_t *v = reinterpret_cast<const CV_G uint32_t *>(G(t.vals) + (size_t)slot * t.vstride);
    mac[0] = v[1]; mac[1] = v[2] & 0xFFFFu;
    node_mac[0] = (v[2] >> 16) | (v[3] << 16); node_mac[1] = v[3] >> 16;
}

// ipcache_lookup4 (eps.h:68-86) -> remote_endpoint_info.sec_label (0 = none)
__device__ __forceinline__ uint32_t ipcache4(const DpParams &p, uint32_t addr_raw, Acct &a)
{
    if (!p.ipc4.l1) return 0;
    a.nl++;
    return lpm4_lookup(p.ipc4, bswap32(addr_raw));
}

// ipcache4 through a quad probe of the /32 front (every lane calls; `want` as in
// quad_find)
__device__ __forceinline__ uint32_t ipcache4_q(const DpParams &p, uint32_t addr_raw, bool want, Acct &a, uint4 *st)
{
    if (!p.ipc4.l1) return 0;
    if (want) a.nl++;
    return lpm4_lookup_q(p.ipc4, bswap32(addr_raw), want, st);
}

// ipcache_lookup6 (eps.h:54-66) at /128
__device__ __forceinline__ uint32_t ipcache6(const DpParams &p, const uint32_t *addr, Acct &a)
{
    if (!p.ipc6.h.buckets) return 0;
    a.nl++;
    return lpm6_lookup(p.ipc6, addr);
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

struct Hit;
__device__ __forceinline__ int policy_hit(const HashTable &pol, uint32_t flags, uint32_t len, int64_t s, bool l4,
                                          uint32_t proxy_port, Acct &a, Hit *defer);

// A policy counter update held back by the lane: the atomic is issued after the
// lane's last dependent lookup, so in-order vmcnt never makes a lookup wait for it.
struct Hit {
    unsigned long long *p;
    unsigned long long inc;
};

__device__ __forceinline__ void hit_flush(const Hit &h)
{
    if (h.p) __hip_atomic_fetch_add(G(h.p), h.inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// __policy_can_access (policy.h:51-119); cb[CB_POLICY] is 0 on these paths.  With
// `defer` the counter update is returned instead of issued.
// With ILP the three keys' buckets are read together (one round trip instead of up
// to three dependent ones; more lines read when an early step hits).  The endpoint
// policy programs use the sequential form: their traffic mostly hits the first (L4)
// key, and the stage measured 6 % faster reading one bucket instead of three.
template <bool ILP = false>
__device__ __forceinline__ int policy_access(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t identity,
                                             uint32_t dport_raw, uint32_t proto, int dir, Acct &a,
                                             Hit *defer = nullptr)
{
    if (flags & F_DROP_ALL) return DROP_POLICY;
    const uint32_t eg = dir ? 0u : 1u;                           // policy_key.egress = !dir
    int64_t s = -1;
    uint32_t px[1] = {0};
    bool l4 = false;
    const uint32_t kl4[2] = {identity, (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24)};
    const uint32_t kl3[2] = {identity, eg << 24};
    const uint32_t kwc[2] = {0, (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24)};
    if constexpr (ILP) {
        const bool have_l4 = flags & F_HAVE_L4_POLICY;
        Probe<PolicySpec> p1, p3;
        if (have_l4) p1 = probe_begin<PolicySpec>(pol, kl4);
        const Probe<PolicySpec> p2 = probe_begin<PolicySpec>(pol, kl3);
        if (have_l4) p3 = probe_begin<PolicySpec>(pol, kwc);
        if (have_l4) {
            a.nl++;
            s = probe_end<PolicySpec>(p1, pol, kl4, px);
            l4 = s >= 0;
        }
        if (s < 0) {
            a.nl++;
            s = probe_end<PolicySpec>(p2, pol, kl3, px);
        }
        if (s < 0 && have_l4) {
            a.nl++;
            s = probe_end<PolicySpec>(p3, pol, kwc, px);
            l4 = s >= 0;
        }
    } else {
        // tag-first probes: the 16-B part with the fingerprints, then the matching
        // key's part (2-3 line requests instead of the whole 64-B bucket's 4 per
        // lane; the config-3 stage 1.5 % faster)
        if (flags & F_HAVE_L4_POLICY) {
            a.nl++;
            s = dev_find_tf<PolicySpec, true>(pol, kl4, px);
            l4 = s >= 0;
        }
        if (s < 0) {
            a.nl++;
            s = dev_find_tf<PolicySpec, true>(pol, kl3, px);
        }
        if (s < 0 && (flags & F_HAVE_L4_POLICY)) {
            a.nl++;
            s = dev_find_tf<PolicySpec, true>(pol, kwc, px);
            l4 = s >= 0;
        }
    }
    return policy_hit(pol, flags, len, s, l4, px[0], a, defer);
}

// the end of __policy_can_access once the lookups are done: slot s (or -1) of the
// matching entry, l4 if it was an L4 key, its inline proxy port
__device__ __forceinline__ int policy_hit(const HashTable &pol, uint32_t flags, uint32_t len, int64_t s, bool l4,
                                          uint32_t proxy_port, Acct &a, Hit *defer)
{
    if (s < 0) return DROP_POLICY;
    a.nu++;
    CV_G uint8_t *v = G(pol.vals) + (size_t)s * pol.vstride;
    // __sync_fetch_and_add(packets, 1) and (bytes, len) as ONE 64-bit atomic on the
    // slot's delta word {count:25 | bytes:39} (launches are chunked to <= 2^24
    // packets and folded after each chunk, so neither field can overflow)
    if (len < (1u << 15)) {
        unsigned long long *d = pol.aux + s;
        const unsigned long long inc = (1ull << 39) | len;
        if (defer) *defer = Hit{d, inc};
        else pol_add(a.pc, d, inc);
    } else {
        __hip_atomic_fetch_add(reinterpret_cast<CV_G unsigned long long *>(v + 8), 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(reinterpret_cast<CV_G unsigned long long *>(v + 16), (unsigned long long)len,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return l4 ? (int)proxy_port : TC_ACT_OK;
}

// policy_access with quad probes (quad_find): every lane of the wave calls it;
// `want` false = this lane does not look up (result unused)
__device__ __forceinline__ int policy_access_q(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t identity,
                                               uint32_t dport_raw, uint32_t proto, int dir, Acct &a, Hit *defer,
                                               bool want, uint4 *st)
{
    want = want && !(flags & F_DROP_ALL);
    const uint32_t eg = dir ? 0u : 1u;
    const bool have_l4 = flags & F_HAVE_L4_POLICY;
    int64_t s = -1;
    uint32_t px = 0, v1 = 0, v2 = 0, v3 = 0;
    bool l4 = false;
    const uint32_t kl4[2] = {identity, (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24)};
    const uint32_t kl3[2] = {identity, eg << 24};
    const uint32_t kwc[2] = {0, (dport_raw & 0xFFFFu) | (proto << 16) | (eg << 24)};
    if (have_l4) {
        const int64_t s1 = quad_find<PolicySpec>(pol, kl4, want, st, &v1);
        if (want) { a.nl++; s = s1; px = v1; l4 = s1 >= 0; }
    }
    const int64_t s2 = quad_find<PolicySpec>(pol, kl3, want && s < 0, st, &v2);
    if (want && s < 0) { a.nl++; s = s2; px = v2; }
    if (have_l4) {
        const int64_t s3 = quad_find<PolicySpec>(pol, kwc, want && s < 0, st, &v3);
        if (want && s < 0) { a.nl++; s = s3; px = v3; l4 = s3 >= 0; }
    }
    if (!want) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
    return policy_hit(pol, flags, len, s, l4, px, a, defer);
}

// policy_ingress through policy_access_q (convergent; `want` as there)
__device__ __forceinline__ int policy_ingress_q(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t src,
                                                uint32_t dport_raw, uint32_t proto, Acct &a, Hit *defer, bool want,
                                                uint4 *st)
{
    const bool look = (flags & F_POLICY_INGRESS) && !(flags & F_DROP_ALL);
    const int r = policy_access_q(pol, flags, len, src, dport_raw, proto, CT_INGRESS, a, defer, want && look, st);
    if (!(flags & F_POLICY_INGRESS)) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
    if (flags & F_DROP_ALL) return DROP_POLICY;
    return r >= TC_ACT_OK ? r : DROP_POLICY;
}

// policy_can_access_ingress (policy.h:139-163)
template <bool ILP = false>
__device__ __forceinline__ int policy_ingress(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t src,
                                              uint32_t dport_raw, uint32_t proto, Acct &a, Hit *defer = nullptr)
{
    if (!(flags & F_POLICY_INGRESS)) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
    if (flags & F_DROP_ALL) return DROP_POLICY;
    int r = policy_access<ILP>(pol, flags, len, src, dport_raw, proto, CT_INGRESS, a, defer);
    return r >= TC_ACT_OK ? r : DROP_POLICY;
}

// policy_can_access_ingress's verdict alone (no counter update, no accounting): true
// when it returns DROP_POLICY
__device__ __forceinline__ bool policy_ingress_denies(const HashTable &pol, uint32_t flags, uint32_t src,
                                                      uint32_t dport_raw, uint32_t proto)
{
    if (!(flags & F_POLICY_INGRESS)) return (flags & F_DROP_ALL) != 0;
    if (flags & F_DROP_ALL) return true;
    uint32_t px[1];
    const uint32_t kl4[2] = {src, (dport_raw & 0xFFFFu) | (proto << 16)};
    const uint32_t kl3[2] = {src, 0u};
    const uint32_t kwc[2] = {0u, (dport_raw & 0xFFFFu) | (proto << 16)};
    const bool l4 = flags & F_HAVE_L4_POLICY;
    if (l4 && dev_find_tf<PolicySpec, true>(pol, kl4, px) >= 0) return false;
    if (dev_find_tf<PolicySpec, true>(pol, kl3, px) >= 0) return false;
    return !(l4 && dev_find_tf<PolicySpec, true>(pol, kwc, px) >= 0);
}

// policy_can_egress (policy.h:181-200), POLICY_EGRESS && LXC_ID.  ILP: the three keys'
// buckets read together; the IPv6 egress stage measured 3.5 % faster with the
// sequential tag-first probes, the IPv4 one 1 % slower.
template <bool ILP = true>
__device__ __forceinline__ int policy_egress(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t identity,
                                             uint32_t dport_raw, uint32_t proto, Acct &a)
{
    if (!(flags & F_POLICY_EGRESS)) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
    if (flags & F_DROP_ALL) return DROP_POLICY;
    int r = policy_access<ILP>(pol, flags, len, identity, dport_raw, proto, CT_EGRESS, a);
    return r >= 0 ? r : DROP_POLICY;
}

// ------------------------------------------------------------------ convergent probes
// The position stages (k_egress_ct, k_egress_deliver) run one packet per lane with every
// lane of a wave at the same call sites (a lane without a packet, or past its drop,
// passes want = false), so their 64-B-bucket lookups are quad probes (cv_hash.hpp): a
// bucket read costs the texture path one line access per lane instead of four.  Q =
// false: the same lookups lane by lane (the continuation list, whose lanes diverge).
template <bool Q, class S>
__device__ __forceinline__ int64_t find_q(const HashTable &t, const uint32_t *key, bool want, uint4 *st, uint32_t *ival)
{
    if constexpr (Q) return quad_find<S>(t, key, want, st, ival);
    else return want ? dev_find<S>(t, key, ival) : -1;
}

// ipcache_lookup4 at /32 of a raw address (0 = no entry); counts the lookup when `want`
template <bool Q>
__device__ __forceinline__ uint32_t ipcache4_at(const DpParams &p, uint32_t addr_raw, bool want, Acct &a, uint4 *st)
{
    if (!p.ipc4.l1) return 0;
    if (want) a.nl++;
    if constexpr (Q) return lpm4_lookup_q(p.ipc4, bswap32(addr_raw), want, st);
    else return want ? lpm4_lookup(p.ipc4, bswap32(addr_raw)) : 0u;
}

// policy_can_egress / policy_can_access_ingress with the convergent probes (`want` as
// in quad_find; the result of a lane without a lookup is meaningless)
template <bool Q>
__device__ __forceinline__ int policy_egress_at(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t identity,
                                                uint32_t dport_raw, uint32_t proto, Acct &a, bool want, uint4 *st)
{
    if constexpr (!Q) {
        if (!want) return DROP_POLICY;
        return policy_egress<true>(pol, flags, len, identity, dport_raw, proto, a);
    } else {
        if (!(flags & F_POLICY_EGRESS)) return (flags & F_DROP_ALL) ? DROP_POLICY : TC_ACT_OK;
        if (flags & F_DROP_ALL) return DROP_POLICY;
        const int r = policy_access_q(pol, flags, len, identity, dport_raw, proto, CT_EGRESS, a, nullptr, want, st);
        return r >= 0 ? r : DROP_POLICY;
    }
}

template <bool Q>
__device__ __forceinline__ int policy_ingress_at(const HashTable &pol, uint32_t flags, uint32_t len, uint32_t src,
                                                 uint32_t dport_raw, uint32_t proto, Acct &a, bool want, uint4 *st)
{
    if constexpr (!Q) {
        if (!want) return DROP_POLICY;
        return policy_ingress<false>(pol, flags, len, src, dport_raw, proto, a);
    } else {
        return policy_ingress_q(pol, flags, len, src, dport_raw, proto, a, nullptr, want, st);
    }
}

__device__ __forceinline__ void store_out(const OutDev &o, uint32_t i, const Acct &a)
{
    if (o.nl) o.nl[i] = (uint8_t)a.nl;
    if (o.nu) o.nu[i] = (uint8_t)a.nu;
}

// ------------------------------------------------------------------ config 1
// check_filters / check_v4 / check_v6 (bpf_xdp.c:88-178)
template <int NW>
__device__ __forceinline__ uint8_t xdp_verdict(const DpParams &p, const RecT<NW> &r, Acct &a)
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

// xdp_verdict with the IPv4 table probes as quad probes (cv_hash.hpp quad_find):
// every lane of the wave calls it (`live` false past the batch end); other frames
// take xdp_verdict's per-lane path, which then does no IPv4 probe.
// *lxc_slot / *lxc_iv (optional): the cilium_lxc probe of an IPv4 daddr, for a caller
// that looks the same key up again in the same table (from_netdev's handle_ipv4)
template <int NW>
__device__ __forceinline__ uint8_t xdp_verdict_q(const DpParams &p, const RecT<NW> &r, Acct &a, bool live,
                                                 uint4 *st, int64_t *lxc_slot = nullptr, uint32_t *lxc_iv = nullptr)
{
    const bool v4 = live && r.len >= 34 && rec_raw16c<12>(r) == 0x0008u;
    uint32_t saddr = rec_raw32c<26>(r), daddr = rec_raw32c<30>(r);
    bool drop = false;
    if (p.cidr4_fix.buckets) {                              // CIDR4_FILTER
        if (p.cidr4_dyn.l1) {                               // CIDR4_LPM_PREFILTER
            if (v4) a.nl++;
            drop = lpm4_lookup_q(p.cidr4_dyn, bswap32(saddr), v4, st) != 0;
        }
        const bool want = v4 && !drop;
        if (want) a.nl++;
        drop = quad_find<Cidr4Spec>(p.cidr4_fix, &saddr, want, st, nullptr) >= 0 || drop;
    }
    uint32_t iv = 0;
    const bool want_lxc = v4 && !drop && p.lxc4.buckets;
    if (want_lxc) a.nl++;
    const int64_t ls = quad_find<LxcV4Spec>(p.lxc4, &daddr, want_lxc, st, &iv);
    const bool hit = ls >= 0;
    if (lxc_slot) { *lxc_slot = ls; *lxc_iv = iv; }
    if (v4) return (!drop && hit) ? XDP_PASS : XDP_DROP;
    if (!live) return XDP_PASS;
    return xdp_verdict(p, r, a);
}

// ------------------------------------------------------------------ conntrack
// struct ct_entry (common.h:380-406) held in 16 words: counters w0-7, lifetime w8,
// bits | rev_nat_index << 16 in w9, slave | tx_flags_seen << 16 | rx_flags_seen << 24
// in w10, src_sec_id w11, last_tx_report w12, last_rx_report w13
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

// struct ct_state (common.h:452-461)
struct CtState {
    uint32_t rev_nat, loopback, slave;
    uint32_t addr, svc_addr, src_sec_id;
};

// Storage of a struct ct_entry (CtE words: w0-7 rx/tx packets/bytes as u64 pairs,
// w8 lifetime, w9 flags | rev_nat << 16, w10 slave | tx/rx_flags_seen, w11 src_sec_id,
// w12/w13 last tx/rx report, w14/15 the slot padding k_nat_apply tags).  A lookup hit
// touches the hot half, kept in the bucket right after the slot's key (CT_HOTW words:
// w8-w13 and the low words of the four counters), so the key and the entry share
// one line; the counters' high words and w14/15 sit in a 32-B side slot, written
// only when a low word carries, at a create, or by the map API.

template <class S>
__device__ __forceinline__ CV_G uint32_t *ct_hot(const HashTable &t, int64_t slot)
{
    static_assert(S::KS >= S::KW + CT_HOTW, "slot holds the hot words");
    return G(t.buckets) + (uint64_t)slot / S::SPB * S::BW + S::KEY0 + (uint32_t)((uint64_t)slot % S::SPB) * S::KS +
           S::KW;
}

template <class S>
__device__ __forceinline__ CV_G uint32_t *ct_cold(const HashTable &t, int64_t slot)
{
    return reinterpret_cast<CV_G uint32_t *>(G(t.vals) + (size_t)slot * CT_COLD);
}

// hot words <-> CtE, the 40-B hot run h0..h9 = {w8 w9 w0 w2 w10 w11 w12 w13 w4 w6} moved
// with three vector accesses (two 16-B, one 8-B) instead of five 8-B ones: the texture
// path spends its cycles per instruction, so every access saved counts for a stage
// bound by line accesses.  A CT6 slot's run starts 16-B aligned (bytes 48 / 128 / 208 of
// its 256-B bucket); a CT4 slot's at byte 24 (slot 0) or 80 (slot 1) of its 128-B bucket:
// the same three instructions for both slots, at per-lane addresses (16-B pair at A,
// 8-B word at B) and a per-lane word order -- no branch, so lanes on either slot issue
// the same instructions.
template <class S>
struct HotAt {
    CV_G uint4 *a;             // 16-B pair start
    CV_G uint2 *b;             // the 8-B part
    bool lo;                   // the 8-B part holds h0, h1 (CT4 slot 0), else h8, h9
};

template <class S>
__device__ __forceinline__ HotAt<S> hot_at(const HashTable &t, int64_t slot)
{
    CV_G uint32_t *h = ct_hot<S>(t, slot);
    static_assert(S::KW == 4 || S::KW == 10, "CT4 / CT6 slots");
    if constexpr (S::KW == 10) {                                  // CT6: 16-B aligned run
        return HotAt<S>{reinterpret_cast<CV_G uint4 *>(h), reinterpret_cast<CV_G uint2 *>(h + 8), false};
    } else {
        const bool s0 = ((uint64_t)slot % S::SPB) == 0;           // run at byte 24: h0 h1 | h2-h5 | h6-h9
        return HotAt<S>{reinterpret_cast<CV_G uint4 *>(s0 ? h + 2 : h), reinterpret_cast<CV_G uint2 *>(s0 ? h : h + 8),
                        s0};
    }
}

// CV_HOT_CONTIG: the run read and written in its memory order (h0-h3, h4-h7, h8-h9) at
// the run's own start -- 8-B aligned for a CT4 slot, so the 16-B accesses there are
// dword-aligned, not 16-B aligned (the global path serves both at one request each) --
// and a hit writes back only the parts whose words changed (ct_store_hot_diff)
#ifndef CV_HOT_CONTIG
#define CV_HOT_CONTIG 1
#endif

template <class S>
__device__ __forceinline__ void ct_load_hot(const HashTable &t, int64_t slot, CtE &e)
{
#if CV_HOT_CONTIG
    {
        const CV_G uint32_t *h = ct_hot<S>(t, slot);
        const uint4 u = *reinterpret_cast<const CV_G uint4 *>(h), v = *reinterpret_cast<const CV_G uint4 *>(h + 4);
        const uint2 w = *reinterpret_cast<const CV_G uint2 *>(h + 8);
        e.w[8] = u.x; e.w[9] = u.y; e.w[0] = u.z; e.w[2] = u.w; e.w[10] = v.x; e.w[11] = v.y;
        e.w[12] = v.z; e.w[13] = v.w; e.w[4] = w.x; e.w[6] = w.y;
        return;
    }
#endif
    const HotAt<S> q = hot_at<S>(t, slot);
    const uint4 u = q.a[0], v = q.a[1];
    const uint2 w = *q.b;
    uint32_t h[10];
    if (q.lo) {
        h[0] = w.x; h[1] = w.y; h[2] = u.x; h[3] = u.y; h[4] = u.z; h[5] = u.w; h[6] = v.x; h[7] = v.y; h[8] = v.z; h[9] = v.w;
    } else {
        h[0] = u.x; h[1] = u.y; h[2] = u.z; h[3] = u.w; h[4] = v.x; h[5] = v.y; h[6] = v.z; h[7] = v.w; h[8] = w.x; h[9] = w.y;
    }
    e.w[8] = h[0]; e.w[9] = h[1]; e.w[0] = h[2]; e.w[2] = h[3]; e.w[10] = h[4]; e.w[11] = h[5];
    e.w[12] = h[6]; e.w[13] = h[7]; e.w[4] = h[8]; e.w[6] = h[9];
}

// NT: the lookup-hit update (ct_hit), written with non-temporal stores -- an entry a
// batch touches once leaves the L2 to the policy tables and endpoint descriptors
#ifndef CV_NT_HIT
#define CV_NT_HIT 0
#endif
typedef uint32_t nt_u4 __attribute__((ext_vector_type(4)));
typedef uint32_t nt_u2 __attribute__((ext_vector_type(2)));

template <class S, bool NT = false>
__device__ __forceinline__ void ct_store_hot(const HashTable &t, int64_t slot, const CtE &e)
{
#if CV_HOT_CONTIG
    if constexpr (!NT) {
        CV_G uint32_t *h = ct_hot<S>(t, slot);
        *reinterpret_cast<CV_G uint4 *>(h) = make_uint4(e.w[8], e.w[9], e.w[0], e.w[2]);
        *reinterpret_cast<CV_G uint4 *>(h + 4) = make_uint4(e.w[10], e.w[11], e.w[12], e.w[13]);
        *reinterpret_cast<CV_G uint2 *>(h + 8) = make_uint2(e.w[4], e.w[6]);
        return;
    }
#endif
    const HotAt<S> q = hot_at<S>(t, slot);
    const uint32_t h[10] = {e.w[8], e.w[9], e.w[0], e.w[2], e.w[10], e.w[11], e.w[12], e.w[13], e.w[4], e.w[6]};
    uint4 u, v;
    uint2 w;
    if (q.lo) {
        w = make_uint2(h[0], h[1]); u = make_uint4(h[2], h[3], h[4], h[5]); v = make_uint4(h[6], h[7], h[8], h[9]);
    } else {
        u = make_uint4(h[0], h[1], h[2], h[3]); v = make_uint4(h[4], h[5], h[6], h[7]); w = make_uint2(h[8], h[9]);
    }
    if constexpr (NT) {
        __builtin_nontemporal_store(nt_u4{u.x, u.y, u.z, u.w}, reinterpret_cast<CV_G nt_u4 *>(q.a));
        __builtin_nontemporal_store(nt_u4{v.x, v.y, v.z, v.w}, reinterpret_cast<CV_G nt_u4 *>(q.a + 1));
        __builtin_nontemporal_store(nt_u2{w.x, w.y}, reinterpret_cast<CV_G nt_u2 *>(q.b));
    } else {
        q.a[0] = u;
        q.a[1] = v;
        *q.b = w;
    }
}

// a hit's write-back: the parts of the run whose words differ from what was loaded (o)
// -- an ingress hit changes h0-h3 alone (lifetime, bits, the rx counters), an egress hit
// h0-h3 and the tx counters, and the flags-seen word and report stamps (h4-h7) change
// once per CT_REPORT_INTERVAL
template <class S>
__device__ __forceinline__ void ct_store_hot_diff(const HashTable &t, int64_t slot, const CtE &e, const CtE &o)
{
#if CV_HOT_CONTIG
    CV_G uint32_t *h = ct_hot<S>(t, slot);
    if ((e.w[8] ^ o.w[8]) | (e.w[9] ^ o.w[9]) | (e.w[0] ^ o.w[0]) | (e.w[2] ^ o.w[2]))
        *reinterpret_cast<CV_G uint4 *>(h) = make_uint4(e.w[8], e.w[9], e.w[0], e.w[2]);
    if ((e.w[10] ^ o.w[10]) | (e.w[11] ^ o.w[11]) | (e.w[12] ^ o.w[12]) | (e.w[13] ^ o.w[13]))
        *reinterpret_cast<CV_G uint4 *>(h + 4) = make_uint4(e.w[10], e.w[11], e.w[12], e.w[13]);
    if ((e.w[4] ^ o.w[4]) | (e.w[6] ^ o.w[6]))
        *reinterpret_cast<CV_G uint2 *>(h + 8) = make_uint2(e.w[4], e.w[6]);
#else
    (void)o;
    ct_store_hot<S, CV_NT_HIT != 0>(t, slot, e);
#endif
}

template <class S>
__device__ __forceinline__ void ct_load(const HashTable &t, int64_t slot, CtE &e)
{
    ct_load_hot<S>(t, slot, e);
    const CV_G uint4 *c = reinterpret_cast<const CV_G uint4 *>(ct_cold<S>(t, slot));
    const uint4 u = c[0], v = c[1];
    e.w[1] = u.x; e.w[3] = u.y; e.w[5] = u.z; e.w[7] = u.w;
    e.w[14] = v.x; e.w[15] = v.y;
}

// cold_known_zero: the slot was just claimed (free slots hold zero side words, see
// dev_kill and k_ct_gc) and e's cold words are zero, so only the bucket line changes
template <class S>
__device__ __forceinline__ void ct_store(const HashTable &t, int64_t slot, const CtE &e, bool cold_known_zero = false)
{
    ct_store_hot<S>(t, slot, e);
    if (cold_known_zero && !(e.w[1] | e.w[3] | e.w[5] | e.w[7] | e.w[14] | e.w[15])) return;
    CV_G uint4 *c = reinterpret_cast<CV_G uint4 *>(ct_cold<S>(t, slot));
    c[0] = make_uint4(e.w[1], e.w[3], e.w[5], e.w[7]);
    c[1] = make_uint4(e.w[14], e.w[15], 0u, 0u);
}

// counter k (0 rx_packets, 2 rx_bytes, 4 tx_packets, 6 tx_bytes) += v on an entry whose
// hot words are loaded: the low word in place, a carry into the side slot's high word
template <class S>
__device__ __forceinline__ void ct_count(const HashTable &t, int64_t slot, CtE &e, int k, uint32_t v)
{
    const uint32_t lo = e.w[k] + v;
    if (lo < e.w[k]) {
        CV_G uint32_t *hi = ct_cold<S>(t, slot) + (k >> 1);
        *hi = *hi + 1u;
    }
    e.w[k] = lo;
}

// The slot as it was before this pass's first write to it (Snap, cv_dp.hpp), into the
// packet's next log entry, part by part: SNAP_HOT its bucket words (tag byte, key, hot
// run), SNAP_COLD its side slot -- a hit changes the hot run alone unless a counter
// carries, so most entries never read the side slot's line.  SNAP_FRESH: the slot was
// just claimed for a new key, `was` its tag before (empty or dead; restored exactly: a
// pass undone as tombstones would lengthen every later miss's probe chain).
enum : uint32_t { SNAP_HOT = 1, SNAP_COLD = 2, SNAP_FRESH = 4 };
template <class S>
__device__ __forceinline__ void snap_slot(const Snap &sn, const HashTable &t, int64_t slot, uint32_t parts, uint32_t was,
                                          Acct &a)
{
    constexpr uint32_t SPARE = S::KEY0 + S::SPB * S::KS;          // (the bucket's first word past its slots)
    static_assert(SPARE < S::BW && S::SPB <= 8, "a CT bucket has a spare word");
    const uint64_t b = (uint64_t)slot / S::SPB;
    const uint32_t s = (uint32_t)((uint64_t)slot % S::SPB);
    CV_G uint32_t *bw = G(t.buckets) + b * S::BW;
    const uint32_t want = ((parts & SNAP_HOT) ? 1u << s : 0u) | ((parts & SNAP_COLD) ? 1u << (8 + s) : 0u);
    const uint32_t prev = __hip_atomic_fetch_or(bw + SPARE, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t hot = (want & ~prev) & (1u << s), cold_new = (want & ~prev) & (1u << (8 + s));
    if (!hot && !cold_new) return;                                // (saved before in this pass)
    if (a.scnt >= SNAP_PER || a.spkt >= sn.n) {                  // (no log entry: the bits go back, so no
        __hip_atomic_fetch_and(bw + SPARE, ~(want & ~prev), __ATOMIC_RELAXED,   //  later pass skips the slot)
                               __HIP_MEMORY_SCOPE_AGENT);
        atomicOr(sn.err, 1u);
        return;
    }
    const bool fresh = parts & SNAP_FRESH;
    const CV_G uint32_t *cold = ct_cold<S>(t, slot);
    uint32_t *d = reinterpret_cast<uint32_t *>(sn.log + ((size_t)a.spkt * SNAP_PER + a.scnt++) * SNAP_U4);
    const unsigned long long ba = (unsigned long long)(uintptr_t)bw, ca = (unsigned long long)(uintptr_t)cold;
    d[0] = (uint32_t)ba;
    d[1] = (uint32_t)(ba >> 32);
    d[32] = (uint32_t)ca;
    d[33] = (uint32_t)(ca >> 32);
    uint32_t tag = 0;
    if (hot) {
        tag = fresh ? was : (bw[s >> 2] >> (8 * (s & 3))) & 0xFFu;
        const CV_G uint32_t *kw = bw + S::KEY0 + s * S::KS;
#pragma unroll 1
        for (int j = 0; j < S::KS; ++j) d[4 + j] = fresh ? 0u : kw[j];
    }
    if (cold_new) {
#pragma unroll 1
        for (int j = 0; j < 8; ++j) d[24 + j] = fresh ? 0u : cold[j];
    }
    d[2] = s | tag << 8 | (uint32_t)S::KS << 16 | SPARE << 24;
    d[3] = (hot ? SNAP_HOT : 0u) | (cold_new ? SNAP_COLD : 0u);
}

template <class S>
__device__ __forceinline__ void snap_before(Acct &a, const HashTable &t, int64_t slot, uint32_t parts,
                                            uint32_t was = TAG_DEAD)
{
    if (a.snap && a.snap->n) snap_slot<S>(*a.snap, t, slot, parts, was, a);
}

// __ct_update_timeout (conntrack.h:103-161): true = report (the `monitor` result)
__device__ __forceinline__ bool ct_timeout_raw(CtE &e, uint32_t lifetime, int dir, uint32_t seen, uint32_t now)
{
    e.w[8] = now + lifetime;
    const int fsh = dir == CT_INGRESS ? 24 : 16;                // rx_flags_seen @43, tx_flags_seen @42
    const int li = dir == CT_INGRESS ? 13 : 12;                 // last_rx_report @52, last_tx_report @48
    const uint32_t acc = (e.w[10] >> fsh) & 0xFFu;
    seen = (seen | acc) & 0xFFu;
    if (e.w[li] + CT_REPORT_INTERVAL < now || acc != seen) {
        e.w[li] = now;
        e.w[10] = (e.w[10] & ~(0xFFu << fsh)) | (seen << fsh);
        return true;
    }
    return false;
}

// ct_update_timeout (conntrack.h:169-186)
__device__ __forceinline__ bool ct_timeout(CtE &e, bool tcp, int dir, uint32_t seen, uint32_t now)
{
    uint32_t lifetime = CT_LIFETIME_NONTCP;
    if (tcp) {
        if (!(seen & TCPF_SYN)) e.set_bits(e.bits() | CTB_SEEN_NON_SYN);
        lifetime = (e.bits() & CTB_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    return ct_timeout_raw(e, lifetime, dir, seen, now);
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
    __device__ void reverse()   // ipv4_ct_tuple_reverse (conntrack.h:414-431)
    {
        uint32_t x = saddr; saddr = daddr; daddr = x;
        x = sport; sport = dport; dport = x;
        flags ^= TUPLE_F_IN;
    }
    static constexpr int KW = 4;
    using Spec = Ct4Spec;
};

struct Tuple6 {                 // struct ipv6_ct_tuple (common.h:338-346), 10 words
    uint32_t daddr[4], saddr[4];
    uint32_t dport, sport;
    uint32_t nexthdr, flags;
    __device__ void key(uint32_t *k) const
    {
#pragma unroll
        for (int j = 0; j < 4; ++j) { k[j] = daddr[j]; k[4 + j] = saddr[j]; }
        k[8] = (dport & 0xFFFFu) | (sport << 16);
        k[9] = nexthdr | (flags << 8);
    }
    __device__ void reverse()   // ipv6_ct_tuple_reverse (conntrack.h:265-285)
    {
#pragma unroll
        for (int j = 0; j < 4; ++j) { uint32_t x = saddr[j]; saddr[j] = daddr[j]; daddr[j] = x; }
        uint32_t x = sport; sport = dport; dport = x;
        flags ^= TUPLE_F_IN;
    }
    static constexpr int KW = 10;
    using Spec = Ct6Spec;
};

enum { ACTION_UNSPEC = 0, ACTION_CREATE = 1, ACTION_CLOSE = 2 };

// __ct_lookup (conntrack.h:199-263) -> CT_NEW / CT_ESTABLISHED; *slot = hit slot;
// a hit fills ct_state's rev_nat_index / loopback / slave
// the entry update of a __ct_lookup hit (conntrack.h:213-258)
template <class S>
__device__ __forceinline__ void ct_hit(const HashTable &ct, int64_t slot, int action, int dir, bool tcp, uint32_t seen,
                                       uint32_t len, uint32_t now, uint32_t flags, CtState *st, Acct &a,
                                       bool *mon = nullptr);

template <class T>
__device__ __forceinline__ int ct_lookup_one(const HashTable &ct, const T &t, int action, int dir, bool tcp,
                                             uint32_t seen, uint32_t len, uint32_t now, uint32_t flags, int64_t &slot,
                                             CtState *st, Acct &a, bool *mon = nullptr)
{
    uint32_t k[T::KW];
    t.key(k);
    a.nl += a.ctu;
    slot = dev_find<typename T::Spec>(ct, k, nullptr);
    if (slot < 0) {
        if (mon) *mon = true;
        return CT_NEW;
    }
    ct_hit<typename T::Spec>(ct, slot, action, dir, tcp, seen, len, now, flags, st, a, mon);
    return CT_ESTABLISHED;
}

// *mon: the `monitor` output of __ct_lookup (report requested), left as is when the
// reference leaves it (a dead entry on a plain lookup).  Reads and writes the hot
// words only (the bucket line the lookup just read).
// the update of a hit entry's words e (ct_hit without its load and store; the hot-run
// fold of k_ct_hot applies it to an entry it holds for a whole chunk); *mon as ct_hit
template <class S>
__device__ __forceinline__ void ct_hit_apply(const HashTable &ct, int64_t slot, CtE &e, int action, int dir, bool tcp,
                                             uint32_t seen, uint32_t len, uint32_t now, uint32_t flags, bool *mon);

template <class S>
__device__ __forceinline__ void ct_hit(const HashTable &ct, int64_t slot, int action, int dir, bool tcp, uint32_t seen,
                                       uint32_t len, uint32_t now, uint32_t flags, CtState *st, Acct &a, bool *mon)
{
    a.nu += a.ctu;
    CtE e;
    ct_load_hot<S>(ct, slot, e);
    if (a.snap) {                                                 // (egress admission, many maps: the parts
        const int k0 = dir == CT_INGRESS ? 0 : 4;                 //  the update writes; the side slot only
        const bool carry = (flags & F_CT_ACCOUNTING) && (e.w[k0] + 1u < e.w[k0] || e.w[k0 + 2] + len < e.w[k0 + 2]);
        snap_before<S>(a, ct, slot, SNAP_HOT | (carry ? SNAP_COLD : 0u));   //  when a counter carries)
    }
    if (st) {
        st->rev_nat = e.w[9] >> 16;
        st->loopback = (e.bits() & CTB_LB_LOOPBACK) ? 1u : 0u;
        st->slave = e.w[10] & 0xFFFFu;
    }
    const CtE e0 = e;
    ct_hit_apply<S>(ct, slot, e, action, dir, tcp, seen, len, now, flags, mon);
    ct_store_hot_diff<S>(ct, slot, e, e0);
}

template <class S>
__device__ __forceinline__ void ct_hit_apply(const HashTable &ct, int64_t slot, CtE &e, int action, int dir, bool tcp,
                                             uint32_t seen, uint32_t len, uint32_t now, uint32_t flags, bool *mon)
{
    bool m = mon ? *mon : false;
    if (ct_alive(e)) m = ct_timeout(e, tcp, dir, seen, now);
    if (flags & F_CT_ACCOUNTING) {
        if (dir == CT_INGRESS) { ct_count<S>(ct, slot, e, 0, 1u); ct_count<S>(ct, slot, e, 2, len); }
        else                   { ct_count<S>(ct, slot, e, 4, 1u); ct_count<S>(ct, slot, e, 6, len); }
    }
    if (action == ACTION_CREATE) {
        if ((e.bits() & CTB_RX_CLOSING) || (e.bits() & CTB_TX_CLOSING)) {
            e.set_bits(e.bits() & ~(CTB_RX_CLOSING | CTB_TX_CLOSING));
            m = ct_timeout(e, tcp, dir, seen, now);
        }
    } else if (action == ACTION_CLOSE) {
        e.set_bits(e.bits() | (dir == CT_INGRESS ? CTB_RX_CLOSING : CTB_TX_CLOSING));
        m = true;
        if (!ct_alive(e)) ct_timeout_raw(e, CT_CLOSE_TIMEOUT, dir, seen, now);
    }
    if (mon) *mon = m;
}

__device__ __forceinline__ uint8_t dir_flags(int dir)
{
    return dir == CT_INGRESS ? TUPLE_F_OUT : dir == CT_EGRESS ? TUPLE_F_IN : TUPLE_F_SERVICE;
}

// The L4 part of ct_lookup4 / ct_lookup6 (conntrack.h:471-530 / 319-374): fills the
// tuple's ports / flags and returns the action, or a DROP code / E_TRUNC (< 0).
template <bool V6, class T>
__device__ __forceinline__ int ct_l4(T &t, const L4Hdr &h, int dir, uint32_t &seen)
{
    t.flags = dir_flags(dir);
    seen = 0;
    const uint32_t icmp = V6 ? 58u : 1u;
    if (t.nexthdr == icmp) {
        if (h.c1) return chk_err(h.c1, DROP_CT_INVALID_HDR);
        t.sport = 0; t.dport = 0;
        const uint32_t type = h.type;
        if (V6 ? (type >= 1 && type <= 4) : (type == 3 || type == 11 || type == 12)) {
            t.flags |= TUPLE_F_RELATED;
            return ACTION_UNSPEC;
        }
        if (type == (V6 ? 129u : 0u)) { t.dport = V6 ? 128u : 8u; return ACTION_UNSPEC; }   // echo reply
        if (type == (V6 ? 128u : 8u)) t.sport = type;                                      // echo request
        return ACTION_CREATE;
    }
    if (t.nexthdr == 6) {
        if (h.c14) return chk_err(h.c14, DROP_CT_INVALID_HDR);
        seen = h.tflags;
        const int action = (seen & (TCPF_RST | TCPF_FIN)) ? ACTION_CLOSE : ACTION_CREATE;
        if (h.c4) return chk_err(h.c4, DROP_CT_INVALID_HDR);
        t.dport = h.p0; t.sport = h.p2;
        return action;
    }
    if (t.nexthdr == 17) {
        if (h.c4) return chk_err(h.c4, DROP_CT_INVALID_HDR);
        t.dport = h.p0; t.sport = h.p2;
        return ACTION_CREATE;
    }
    return DROP_CT_UNKNOWN_PROTO;
}

// ct_lookup4 / ct_lookup6 (conntrack.h:442-562 / 286-412); tuple in/out
// Both lookup keys are known before the first probe, so the reverse-direction
// probe is issued together with the first one (its result is used only when the
// first misses, as the reference's second __ct_lookup).
// ONE: a single call site for the entry update (the lanes of a wave take different
// branches; the update's loads and stores then issue once for all of them): measured
// 7 % faster in the IPv6 egress stage, 2 % slower in the netdev policy stage.
template <bool V6, bool FRESH = true, bool ONE = false, class T>
__device__ __forceinline__ int ct_lookup(const HashTable &ct, T &t, const L4Hdr &h, int dir, uint32_t len,
                                         uint32_t now, uint32_t flags, int64_t &slot, CtState *st, Acct &a,
                                         bool *mon = nullptr)
{
    using S = typename T::Spec;
    uint32_t seen;
    const int action = ct_l4<V6>(t, h, dir, seen);
    if (action < 0) return action;
    const bool tcp = t.nexthdr == 6;
    T t2 = t;
    t2.reverse();
    uint32_t k1[T::KW], k2[T::KW];
    t.key(k1);
    t2.key(k2);
    const Probe<S> p1 = probe_begin<S, FRESH>(ct, k1);
    Probe<S> p2;
    if (dir != CT_SERVICE) {
        if constexpr (S::SYM != 0) {                              // the reverse tuple's home bucket is the
            p2 = p1;                                              // same (home_hash): one tag read serves both
            p2.tag = tag_of(key_hash<S>(k2));
        } else {
            p2 = probe_begin<S, FRESH>(ct, k2);
        }
    }
    a.nl += a.ctu;
    slot = probe_end<S, FRESH>(p1, ct, k1, nullptr);
    if constexpr (ONE) {
        const bool first = slot >= 0;
        if (!first) {
            if (mon) *mon = true;                                 // the first __ct_lookup missed
            if (dir == CT_SERVICE) return CT_NEW;
            t = t2;
            a.nl += a.ctu;
            slot = probe_end<S, FRESH>(p2, ct, k2, nullptr);
            if (slot < 0) return CT_NEW;
        }
        ct_hit<S>(ct, slot, action, dir, tcp, seen, len, now, flags, st, a, mon);
        if (!first) return CT_ESTABLISHED;
        return (t.flags & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
    }
    if (slot >= 0) {
        ct_hit<S>(ct, slot, action, dir, tcp, seen, len, now, flags, st, a, mon);
        return (t.flags & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
    }
    if (mon) *mon = true;                                         // the first __ct_lookup missed
    if (dir == CT_SERVICE) return CT_NEW;
    t = t2;
    a.nl += a.ctu;
    slot = probe_end<S, FRESH>(p2, ct, k2, nullptr);
    if (slot < 0) return CT_NEW;
    ct_hit<S>(ct, slot, action, dir, tcp, seen, len, now, flags, st, a, mon);
    return CT_ESTABLISHED;
}

// A hit whose entry update is deferred (k_ct_hot's fold applies it in member order)
struct HitRec {
    int64_t slot;              // -1: no hit
    uint32_t action, dir, tcp, seen, len;
};

// ct_lookup4 (conntrack.h:442-562) for the hot-run path: the lookups and the result
// only -- what the entry's hit fields give ct_state (rev_nat_index, loopback, slave)
// -- with the hit's update returned in hr instead of written; accounting as ct_lookup
template <class T>
__device__ __forceinline__ int ct_lookup_pre(const HashTable &ct, T &t, const L4Hdr &h, int dir, uint32_t len,
                                             int64_t &slot, CtState *st, Acct &a, HitRec &hr)
{
    using S = typename T::Spec;
    static_assert(S::SYM != 0, "conntrack");
    uint32_t seen;
    hr.slot = -1;
    slot = -1;
    const int action = ct_l4<T::KW == 10>(t, h, dir, seen);
    if (action < 0) return action;
    T t2 = t;
    t2.reverse();
    uint32_t k1[T::KW], k2[T::KW];
    t.key(k1);
    t2.key(k2);
    int ret;
    a.nl += a.ctu;
    slot = dev_find<S, false>(ct, k1, nullptr);
    if (slot >= 0) {
        ret = (t.flags & TUPLE_F_RELATED) ? CT_RELATED : CT_REPLY;
    } else {
        if (dir == CT_SERVICE) return CT_NEW;
        t = t2;
        a.nl += a.ctu;
        slot = dev_find<S, false>(ct, k2, nullptr);
        if (slot < 0) return CT_NEW;
        ret = CT_ESTABLISHED;
    }
    a.nu += a.ctu;
    const CV_G uint32_t *hw = ct_hot<S>(ct, slot);                 // hot words h1 = w9, h4 = w10
    const uint32_t w9 = hw[1], w10 = hw[4];
    if (st) {
        st->rev_nat = w9 >> 16;
        st->loopback = (w9 & CTB_LB_LOOPBACK) ? 1u : 0u;
        st->slave = w10 & 0xFFFFu;
    }
    hr = HitRec{slot, (uint32_t)action, (uint32_t)dir, t.nexthdr == 6 ? 1u : 0u, seen, len};
    return ret;
}

// The live-entry count of a CT map (its max_entries check).  A launch either has room
// for every create it can make (the host plans launch chunks by the worst case per
// packet, cv_ctx.cpp ct_plan): creates then only count, summed per workgroup in the
// LDS counter cache; or it is a guarded one-packet launch next to the limit, where a
// create of a new key first checks the count, exactly as the kernel's hash map fails
// an insert past max_entries (-E2BIG -> DROP_CT_CREATE_FAILED).
__device__ __forceinline__ void ct_live_add(const HashTable &ct, Acct &a, bool guard, long long d)
{
    if (!ct.live) return;
    if (guard) __hip_atomic_fetch_add(G(ct.live), (unsigned long long)d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else live_add(a.pc, ct.live, (unsigned long long)d);
}

// map_update_elem(BPF_ANY) of a CT entry (conntrack.h:694,720,740)
template <class T>
__device__ __forceinline__ bool ct_put(const HashTable &ct, const T &t, const CtE &e, Acct &a, bool guard,
                                       bool absent = false)
{
    uint32_t k[T::KW];
    t.key(k);
    if (guard && ct.live && (absent || dev_find<typename T::Spec>(ct, k, nullptr) < 0) &&
        __hip_atomic_load(G(ct.live), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ct.cap)
        return false;                                             // full: -E2BIG
    if (a.budget != ~0u && (absent || dev_find<typename T::Spec>(ct, k, nullptr) < 0)) {
        ++a.tried;
        if (!a.budget) return false;                              // admission: the map is full here (-E2BIG)
        --a.budget;
    }
    bool created;
    uint32_t was = TAG_DEAD;
    const int64_t s = dev_upsert<typename T::Spec>(ct, k, &created, absent, &was);
    if (s < 0) return false;
    snap_before<typename T::Spec>(a, ct, s, SNAP_HOT | SNAP_COLD | (created ? SNAP_FRESH : 0u), was);
    if (created) ct_live_add(ct, a, guard, 1);
    ct_store<typename T::Spec>(ct, s, e, created);
    return true;
}

// ct_delete4 / ct_delete6 (conntrack.h:641-647, 564-570) of a found entry
template <class S>
__device__ __forceinline__ void ct_kill(const HashTable &ct, int64_t slot, Acct &a, bool guard)
{
    snap_before<S>(a, ct, slot, SNAP_HOT | SNAP_COLD);
    dev_kill<S>(ct, slot);
    ct_live_add(ct, a, guard, -1);
    a.nu += a.ctu;
    a.killed++;
}

// the entry ct_create4 / ct_create6 write for `t` (conntrack.h:668-690 / 593-612)
__device__ __forceinline__ void ct_entry_new(CtE &e, bool tcp, uint32_t len, int dir, const CtState &st, uint32_t now)
{
#pragma unroll
    for (int k = 0; k < 16; ++k) e.w[k] = 0;
    e.w[9] = (st.rev_nat & 0xFFFFu) << 16 | (st.loopback ? CTB_LB_LOOPBACK : 0u);
    e.w[10] = st.slave & 0xFFFFu;
    ct_timeout(e, tcp, dir, tcp ? TCPF_SYN : 0u, now);
    if (dir == CT_INGRESS) { e.w[0] = 1; e.w[2] = len; }
    else                   { e.w[4] = 1; e.w[6] = len; }
    e.w[11] = st.src_sec_id;
}

// the NATed tuple ct_create4 writes when ct_state->addr is set (conntrack.h:697-725)
__device__ __forceinline__ Tuple4 ct_nat_tuple(const Tuple4 &t, int dir, const CtState &st)
{
    Tuple4 n = t;
    if (dir == CT_INGRESS) n.saddr = st.addr; else n.daddr = st.addr;
    if (st.loopback) {
        n.flags = TUPLE_F_IN;
        if (dir == CT_INGRESS) n.daddr = st.svc_addr; else n.saddr = st.svc_addr;
    }
    return n;
}

// ct_create4 / ct_create6 (conntrack.h:663-744 / 589-639): the entry, the NATed
// tuple when ct_state->addr is set (v4 only; with defer_nat the caller writes it
// later, see k_nat_apply), and the ICMP-RELATED twin.  absent: `t` is the tuple
// ct_lookup just missed (both directions), so its insert skips the key compare.
template <bool V6, class T>
__device__ __forceinline__ int ct_create(const HashTable &ct, const T &t, uint32_t len, int dir, const CtState &st,
                                         uint32_t now, Acct &a, bool guard, bool defer_nat = false,
                                         bool absent = false)
{
    CtE e;
    const bool tcp = t.nexthdr == 6;
    ct_entry_new(e, tcp, len, dir, st, now);
    const bool nat = !V6 && st.addr;
    a.nu += (nat ? 3u : 2u) * a.ctu;
    if (!ct_put(ct, t, e, a, guard, absent)) return DROP_CT_CREATE_FAILED;
    if constexpr (!V6) {
        if (nat && !defer_nat) {
            if (!ct_put(ct, ct_nat_tuple(t, dir, st), e, a, guard)) return DROP_CT_CREATE_FAILED;
        }
    }
    T it = t;
    it.nexthdr = V6 ? 58u : 1u;
    it.sport = 0; it.dport = 0;
    it.flags = t.flags | TUPLE_F_RELATED;
    e.set_bits(e.bits() | CTB_SEEN_NON_SYN);
    if (!ct_put(ct, it, e, a, guard)) return DROP_CT_CREATE_FAILED;
    return 0;
}

// ------------------------------------------------------------------ reverse NAT
// cilium_lb4_reverse_nat / cilium_lb6_reverse_nat lookups (lb.h:562-576, 305-315):
// dense tables indexed by the raw u16 key
__device__ __forceinline__ bool revnat4(const DpParams &p, uint32_t index, uint32_t &addr, uint32_t &port, Acct &a)
{
    if (!p.revnat4) return false;
    a.nl++;
    const uint2 v = reinterpret_cast<const uint2 *>(p.revnat4)[index & 0xFFFFu];
    if (!(v.y >> 16)) return false;
    addr = v.x;
    port = v.y & 0xFFFFu;
    return true;
}

__device__ __forceinline__ bool revnat6(const DpParams &p, uint32_t index, uint32_t *addr, uint32_t &port, Acct &a)
{
    if (!p.revnat6) return false;
    a.nl++;
    const uint4 *q = reinterpret_cast<const uint4 *>(p.revnat6) + 2 * (size_t)(index & 0xFFFFu);
    const uint4 v0 = q[0], v1 = q[1];
    if (!(v1.x >> 16)) return false;
    addr[0] = v0.x; addr[1] = v0.y; addr[2] = v0.z; addr[3] = v0.w;
    port = v1.x & 0xFFFFu;
    return true;
}

// reverse_map_l4_port (lb.h:222-252) inside __lb{4,6}_rev_nat: 0 or a code
__device__ __forceinline__ int rev_map_port(L4Hdr &h, uint32_t nexthdr, uint32_t port)
{
    if (!port) return 0;
    if (nexthdr == 6 || nexthdr == 17) {
        if (h.c2a) return chk_err(h.c2a, E_FAULT);
        if (port != h.p0) h.p0 = port;               // l4_modify_port(TCP_SPORT_OFF)
        return 0;
    }
    if (nexthdr == 1 || nexthdr == 58) return 0;
    return DROP_UNKNOWN_L4;
}

// ------------------------------------------------------------------ the skb after rewrites
struct Skb4 {
    uint32_t saddr, daddr, len, nexthdr, ttl;
    int l4off;
    uint32_t avail;             // bytes of the frame in the record (loads past it: E_TRUNC)
    L4Hdr h;
};

// The L4 checksum update every IPv4 rewrite ends with (csum_l4_offset_and_flags,
// csum.h:44-64: TCP check @16, UDP @6, none for ICMP): 0, or the code of the
// helper's failed access to the field (DROP_CSUM_L4 past the packet, E_TRUNC past
// the record).
__device__ __forceinline__ int l4_csum_err(const Skb4 &s, uint32_t nexthdr)
{
    const int coff = nexthdr == 6 ? 16 : nexthdr == 17 ? 6 : 0;
    if (!coff) return 0;
    const uint32_t end = (uint32_t)(s.l4off + coff + 2);
    if (s.l4off + coff < 0 || end > s.len) return DROP_CSUM_L4;
    if (end > s.avail) return E_TRUNC;
    return 0;
}

struct Skb6 {
    uint32_t saddr[4], daddr[4];
    uint32_t len, nexthdr, hoplimit;
    int l4off;                  // ETH_HLEN + ipv6_hdrlen, or the (negative) ipv6_hdrlen error
    uint32_t avail;             // bytes of the frame in the record
    L4Hdr h;
};

// csum_l4_offset_and_flags (csum.h:44-64) for an IPv6 packet: TCP 16, UDP 6, ICMPv6 2;
// other protocols leave it 0 and the IPv6 rewrites (which do not test it) update the
// field at l4_off + 0
__device__ __forceinline__ int l4_coff6(uint32_t nexthdr)
{
    return nexthdr == 6 ? 16 : nexthdr == 17 ? 6 : nexthdr == 58 ? 2 : 0;
}

// the L4 checksum access of an IPv6 rewrite (lb6_xlate, __lb6_rev_nat, the rev-NAT
// index zeroing of ipv6_policy): 0, DROP_CSUM_L4 past the packet, E_TRUNC past the record
__device__ __forceinline__ int l4_csum_err6(const Skb6 &s)
{
    const uint32_t end = (uint32_t)(s.l4off + l4_coff6(s.nexthdr) + 2);
    if (end > s.len) return DROP_CSUM_L4;
    if (end > s.avail) return E_TRUNC;
    return 0;
}

// ipv6_hdrlen (ipv6.h:61-98): returns the IPv6 header length or a DROP code and
// the final next header.  The AUTH length is chosen by the type of the header that
// FOLLOWS (nh is updated first), as the reference does.
template <int NW>
__device__ __forceinline__ int ipv6_hdrlen(const RecT<NW> &r, uint32_t &nexthdr)
{
    int len = 40;
    uint32_t nh = rec_u8c<20>(r);
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        if (nh == 59) return DROP_INVALID_EXTHDR;
        if (nh == 44) return DROP_FRAG_NOSUPPORT;
        if (nh == 0 || nh == 43 || nh == 51 || nh == 60) {
            const int off = 14 + len;
            const int c = rec_chk(r, off, 2);
            if (c) return chk_err(c, DROP_INVALID);
            const uint32_t b0 = off == 54 ? rec_u8c<54>(r) : r.base[off];
            const uint32_t b1 = off == 54 ? rec_u8c<55>(r) : r.base[off + 1];
            nh = b0;
            len += nh == 51 ? (int)((b1 + 2) << 2) : (int)((b1 + 1) << 3);
            continue;
        }
        nexthdr = nh;
        return len;
    }
    return DROP_INVALID_EXTHDR;
}

__device__ __forceinline__ Skb6 skb6_from(const Rec6 &r)
{
    Skb6 s;
    s.saddr[0] = rec_raw32c<22>(r); s.saddr[1] = rec_raw32c<26>(r); s.saddr[2] = rec_raw32c<30>(r); s.saddr[3] = rec_raw32c<34>(r);
    s.daddr[0] = rec_raw32c<38>(r); s.daddr[1] = rec_raw32c<42>(r); s.daddr[2] = rec_raw32c<46>(r); s.daddr[3] = rec_raw32c<50>(r);
    s.len = r.len;
    s.hoplimit = rec_u8c<21>(r);
    uint32_t nh = rec_u8c<20>(r);
    const int hl = ipv6_hdrlen(r, nh);
    s.nexthdr = nh;
    s.l4off = hl < 0 ? hl : 14 + hl;
    s.avail = r.stride;
    if (hl >= 0) s.h = l4_read<54>(r, s.l4off);
    return s;
}

__device__ __forceinline__ Skb4 skb4_from(const Rec &r)
{
    Skb4 s;
    s.saddr = rec_raw32c<26>(r);
    s.daddr = rec_raw32c<30>(r);
    s.len = r.len;
    s.nexthdr = rec_u8c<23>(r);
    s.ttl = rec_u8c<22>(r);
    s.l4off = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
    s.avail = r.stride;
    s.h = l4_read<34>(r, s.l4off);
    return s;
}

// The stage record of an IPv4 packet that reaches the policy program: the fields
// tail_ipv4_policy reads, packed by the front kernel into 16 B next to the packet's
// hand-over words (StageRec), so stage 2 loads one 32-B slot per packet instead of the
// 64-B record and separate meta / label arrays.  Access outcomes: 2 bits each
// (0 ok, 1 past the packet, 2 past the record -> E_TRUNC).
__device__ __forceinline__ uint32_t chk2(int c) { return c == 0 ? 0u : c == E_TRUNC ? 2u : 1u; }
__device__ __forceinline__ int8_t unchk2(uint32_t v) { return (int8_t)(v == 0 ? 0 : v == 2 ? E_TRUNC : 1); }

__device__ __forceinline__ uint4 skb4_pack(const Skb4 &s, uint32_t &w4, uint32_t &chk)
{
    w4 = (s.nexthdr & 0xFFu) | (s.h.type & 0xFFu) << 8 | (s.h.tflags & 0xFFu) << 16 | (uint32_t)s.l4off << 24;
    chk = chk2(s.h.c1) | chk2(s.h.c14) << 2 | chk2(s.h.c4) << 4 | chk2(s.h.c2a) << 6 | chk2(s.h.c2b) << 8;
    return make_uint4(s.saddr, s.daddr, (s.h.p0 & 0xFFFFu) | s.h.p2 << 16, s.len);
}

__device__ __forceinline__ Skb4 skb4_unpack(const uint4 &a, uint32_t w4, uint32_t chk, uint32_t stride)
{
    Skb4 s;
    s.saddr = a.x;
    s.daddr = a.y;
    s.len = a.w;
    s.nexthdr = w4 & 0xFFu;
    s.ttl = 0;                                                    // (not read after the front)
    s.l4off = (int)(w4 >> 24);
    s.avail = stride;
    s.h.type = (w4 >> 8) & 0xFFu;
    s.h.tflags = (w4 >> 16) & 0xFFu;
    s.h.p0 = a.z & 0xFFFFu;
    s.h.p2 = a.z >> 16;
    s.h.c1 = unchk2(chk & 3u);
    s.h.c14 = unchk2((chk >> 2) & 3u);
    s.h.c4 = unchk2((chk >> 4) & 3u);
    s.h.c2a = unchk2((chk >> 6) & 3u);
    s.h.c2b = unchk2((chk >> 8) & 3u);
    return s;
}

// ------------------------------------------------------------------ output frames (IPv4)
// The frame rewrites of the reference (lb4_xlate lb.h:653-697, __lb4_rev_nat
// lb.h:485-548, ipv4_l3 l3.h:54-69) replayed on the record's fields with the
// kernel's checksum arithmetic (bpf_l3/l4_csum_replace, bpf_csum_diff for
// CHECKSUM_NONE skbs; restated in oracle/cv_oracle.c and pinned there by
// tests/golden/csum_kernel.npz).  Values are memory-order (LE loads of the bytes).
__device__ __forceinline__ uint32_t cs_add(uint32_t a, uint32_t b) { const uint32_t r = a + b; return r + (r < b); }
__device__ __forceinline__ uint32_t cs_fold(uint32_t x)
{
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return ~x & 0xFFFFu;
}
__device__ __forceinline__ uint32_t cs16_add(uint32_t a, uint32_t b)
{
    const uint32_t r = (a + b) & 0xFFFFu;
    return (r + (r < b)) & 0xFFFFu;
}
__device__ __forceinline__ uint32_t csum_diff4(uint32_t from, uint32_t to, uint32_t seed)
{
    uint64_t t = (uint64_t)seed + ((uint64_t)(~from) | ((uint64_t)to << 32));
    if (t < (uint64_t)seed) t++;
    const uint64_t r = (t >> 32) + (t & 0xFFFFFFFFu);
    uint32_t x = (uint32_t)r + (uint32_t)(r >> 32);
    x = (x & 0xFFFFu) + (x >> 16);
    return (x & 0xFFFFu) + (x >> 16);
}
__device__ __forceinline__ uint32_t l3_by_diff(uint32_t c, uint32_t diff) { return cs_fold(cs_add(diff, ~c)); }
__device__ __forceinline__ uint32_t l3_replace2(uint32_t c, uint32_t from, uint32_t to)
{
    return ~cs16_add(cs16_add(~c & 0xFFFFu, ~from & 0xFFFFu), to) & 0xFFFFu;
}
// bpf_l4_csum_replace: size 0 (diff in `to`) or 2; mm = BPF_F_MARK_MANGLED_0 (UDP)
__device__ __forceinline__ uint32_t l4_replace(uint32_t c, uint32_t from, uint32_t to, int size, bool mm)
{
    if (mm && !c) return 0u;
    uint32_t n = size == 0 ? cs_fold(cs_add(to, ~c)) : cs_fold(cs_add(cs_add(~c, ~(from & 0xFFFFu)), to & 0xFFFFu));
    if (mm && !n) n = 0xFFFFu;
    return n;
}

// a __lb4_rev_nat a program applied: {na, np} of the reverse NAT entry
struct RevNatOut {
    bool valid, loopback;
    uint32_t na, np;
};

struct Frame4 {
    uint32_t saddr, daddr, sp, dp, ttl, ipcs, l4cs;
    uint32_t smac[2], dmac[2];
    uint32_t nexthdr;
    int l4off, coff;           // coff 0: no L4 checksum (ICMP, others)
    bool mm, smac_set, dmac_set;
};

// the record as the program sees it before any rewrite; `csum_at` = the frame bytes
// in global memory (the L4 checksum sits at a runtime offset)
template <int NW>
__device__ __forceinline__ void frame4_init(Frame4 &f, const RecT<NW> &r, const uint8_t *frame)
{
    f.saddr = rec_raw32c<26>(r);
    f.daddr = rec_raw32c<30>(r);
    f.ttl = rec_u8c<22>(r);
    f.ipcs = rec_raw16c<24>(r);
    f.nexthdr = rec_u8c<23>(r);
    f.l4off = 14 + (int)(rec_u8c<14>(r) & 0xFu) * 4;
    f.coff = f.nexthdr == 6 ? 16 : f.nexthdr == 17 ? 6 : 0;
    f.mm = f.nexthdr == 17;
    const uint32_t lim = r.len < r.stride ? r.len : r.stride;
    const bool ports = (uint32_t)f.l4off + 4 <= lim;
    f.sp = ports ? (uint32_t)frame[f.l4off] | (uint32_t)frame[f.l4off + 1] << 8 : 0u;
    f.dp = ports ? (uint32_t)frame[f.l4off + 2] | (uint32_t)frame[f.l4off + 3] << 8 : 0u;
    const int co = f.l4off + f.coff;
    f.l4cs = (f.coff && (uint32_t)co + 2 <= lim) ? ((uint32_t)frame[co] | (uint32_t)frame[co + 1] << 8) : 0u;
    f.smac_set = f.dmac_set = false;
}

// lb4_xlate: daddr (and the loopback saddr), their diff into both checksums, the port
__device__ __forceinline__ void frame4_xlate(Frame4 &f, uint32_t vip, uint32_t new_daddr, uint32_t new_saddr,
                                             bool port_rw, uint32_t key_dport, uint32_t new_port)
{
    uint32_t sum = csum_diff4(vip, new_daddr, 0);
    f.daddr = new_daddr;
    if (new_saddr) { sum = csum_diff4(f.saddr, new_saddr, sum); f.saddr = new_saddr; }
    f.ipcs = l3_by_diff(f.ipcs, sum);
    if (f.coff) f.l4cs = l4_replace(f.l4cs, 0, sum, 0, f.mm);
    if (port_rw) {                                                // l4_modify_port(TCP_DPORT_OFF)
        if (f.coff) f.l4cs = l4_replace(f.l4cs, key_dport, new_port, 2, f.mm);
        f.dp = new_port;
    }
}

// __lb4_rev_nat with the reverse NAT entry {na, np}; old_sip = the tuple's saddr
// (REV_NAT_F_TUPLE_SADDR) or the packet's
__device__ __forceinline__ void frame4_revnat(Frame4 &f, uint32_t na, uint32_t np, bool loopback, uint32_t old_sip)
{
    if (np && (f.nexthdr == 6 || f.nexthdr == 17) && np != f.sp) {   // reverse_map_l4_port
        if (f.coff) f.l4cs = l4_replace(f.l4cs, f.sp, np, 2, f.mm);
        f.sp = np;
    }
    uint32_t sum = 0;
    if (loopback) { sum = csum_diff4(f.daddr, old_sip, 0); f.daddr = old_sip; }
    sum = csum_diff4(old_sip, na, sum);
    f.saddr = na;
    f.ipcs = l3_by_diff(f.ipcs, sum);
    if (f.coff) f.l4cs = l4_replace(f.l4cs, 0, sum, 0, f.mm);
}

// ipv4_l3: ipv4_dec_ttl, then the MACs (smac optional)
__device__ __forceinline__ void frame4_l3(Frame4 &f, const uint32_t *smac, const uint32_t *dmac)
{
    const uint32_t nt = (f.ttl - 1) & 0xFFu;
    f.ipcs = l3_replace2(f.ipcs, f.ttl, nt);
    f.ttl = nt;
    if (smac) { f.smac[0] = smac[0]; f.smac[1] = smac[1]; f.smac_set = true; }
    f.dmac[0] = dmac[0]; f.dmac[1] = dmac[1]; f.dmac_set = true;
}

// out = the input record with the rewritten fields
__device__ __forceinline__ void frame4_emit(const Frame4 &f, const uint8_t *in, uint8_t *out, uint32_t stride,
                                            uint32_t len)
{
    const uint32_t lim = len < stride ? len : stride;
    for (uint32_t k = 0; k < stride; k += 16)
        *reinterpret_cast<uint4 *>(out + k) = *reinterpret_cast<const uint4 *>(in + k);
    auto put16 = [&](int off, uint32_t v) { out[off] = (uint8_t)v; out[off + 1] = (uint8_t)(v >> 8); };
    auto put32 = [&](int off, uint32_t v) { put16(off, v & 0xFFFFu); put16(off + 2, v >> 16); };
    if (f.dmac_set) { put32(0, f.dmac[0]); put16(4, f.dmac[1]); }
    if (f.smac_set) { put32(6, f.smac[0]); put16(10, f.smac[1]); }
    out[22] = (uint8_t)f.ttl;
    put16(24, f.ipcs);
    put32(26, f.saddr);
    put32(30, f.daddr);
    if ((uint32_t)f.l4off + 4 <= lim) { put16(f.l4off, f.sp); put16(f.l4off + 2, f.dp); }
    if (f.coff && (uint32_t)(f.l4off + f.coff) + 2 <= lim) put16(f.l4off + f.coff, f.l4cs);
}

__device__ __forceinline__ void frame_copy(const uint8_t *in, uint8_t *out, uint32_t stride)
{
    for (uint32_t k = 0; k < stride; k += 16)
        *reinterpret_cast<uint4 *>(out + k) = *reinterpret_cast<const uint4 *>(in + k);
}

// ------------------------------------------------------------------ output frames (IPv6)
// lb6_xlate (lb.h:398-424), __lb6_rev_nat (lb.h:254-290), ipv6_policy's rev-NAT index
// zeroing (bpf_lxc.c:754-772), ipv6_l3 (l3.h:30-51) and pass_to_stack's
// ipv6_store_flowlabel (ipv6.h:245-260).  No L3 checksum; the L4 one changes by the
// 16-byte bpf_csum_diff of the address (pinned by tests/golden/csum16_kernel.npz).
__device__ __forceinline__ uint32_t csum_diff16(const uint32_t *from, const uint32_t *to, uint32_t seed)
{
    uint64_t t = seed;
#pragma unroll
    for (int j = 0; j < 4; ++j) { t += (uint32_t)~from[j]; t += to[j]; }
    t = (t & 0xFFFFFFFFu) + (t >> 32);
    uint32_t x = (uint32_t)t + (uint32_t)(t >> 32);
    x = (x & 0xFFFFu) + (x >> 16);
    return (x & 0xFFFFu) + (x >> 16);
}

struct RevNat6Out {             // a __lb6_rev_nat a program applied
    bool valid;
    uint32_t na[4], np;
};

struct Frame6 {
    uint32_t saddr[4], daddr[4], w0, hop, sp, dp, l4cs;
    uint32_t smac[2], dmac[2];
    uint32_t nexthdr;
    int l4off, coff;
    bool mm, ports, csum, smac_set, dmac_set;
};

template <int NW>
__device__ __forceinline__ void frame6_init(Frame6 &f, const RecT<NW> &r, int l4off, uint32_t nexthdr,
                                            const uint8_t *frame)
{
    f.saddr[0] = rec_raw32c<22>(r); f.saddr[1] = rec_raw32c<26>(r); f.saddr[2] = rec_raw32c<30>(r); f.saddr[3] = rec_raw32c<34>(r);
    f.daddr[0] = rec_raw32c<38>(r); f.daddr[1] = rec_raw32c<42>(r); f.daddr[2] = rec_raw32c<46>(r); f.daddr[3] = rec_raw32c<50>(r);
    f.w0 = rec_raw32c<14>(r);
    f.hop = rec_u8c<21>(r);
    f.nexthdr = nexthdr;
    f.l4off = l4off;
    f.coff = l4_coff6(nexthdr);
    f.mm = nexthdr == 17;
    const uint32_t lim = r.len < r.stride ? r.len : r.stride;
    f.ports = l4off >= 0 && (uint32_t)l4off + 4 <= lim;
    f.sp = f.ports ? (uint32_t)frame[l4off] | (uint32_t)frame[l4off + 1] << 8 : 0u;
    f.dp = f.ports ? (uint32_t)frame[l4off + 2] | (uint32_t)frame[l4off + 3] << 8 : 0u;
    const int co = l4off + f.coff;
    f.csum = l4off >= 0 && (uint32_t)co + 2 <= lim;
    f.l4cs = f.csum ? ((uint32_t)frame[co] | (uint32_t)frame[co + 1] << 8) : 0u;
    f.smac_set = f.dmac_set = false;
}

// lb6_xlate: daddr, the L4 checksum by the address diff, then l4_modify_port(TCP_DPORT_OFF)
__device__ __forceinline__ void frame6_xlate(Frame6 &f, const uint32_t *target, bool port_rw, uint32_t key_dport,
                                             uint32_t new_port)
{
    f.l4cs = l4_replace(f.l4cs, 0, csum_diff16(f.daddr, target, 0), 0, f.mm);
#pragma unroll
    for (int j = 0; j < 4; ++j) f.daddr[j] = target[j];
    if (port_rw) { f.l4cs = l4_replace(f.l4cs, key_dport, new_port, 2, f.mm); f.dp = new_port; }
}

// __lb6_rev_nat(flags 0): reverse_map_l4_port, then the packet's saddr and its diff
__device__ __forceinline__ void frame6_revnat(Frame6 &f, const RevNat6Out &rn)
{
    if (rn.np && (f.nexthdr == 6 || f.nexthdr == 17) && rn.np != f.sp) {
        f.l4cs = l4_replace(f.l4cs, f.sp, rn.np, 2, f.mm);
        f.sp = rn.np;
    }
    f.l4cs = l4_replace(f.l4cs, 0, csum_diff16(f.saddr, rn.na, 0), 0, f.mm);
#pragma unroll
    for (int j = 0; j < 4; ++j) f.saddr[j] = rn.na[j];
}

// ipv6_policy: rev_nat_index = the low 16 bits of daddr word 3, zeroed in the packet,
// checksum by csum_diff(&rev_nat_index, 4, &zero, 4, 0) when the L4 has a checksum offset
__device__ __forceinline__ void frame6_zero_revnat(Frame6 &f)
{
    const uint32_t rni = f.daddr[3] & 0xFFFFu;
    if (!rni) return;
    f.daddr[3] &= ~0xFFFFu;
    if (f.coff) f.l4cs = l4_replace(f.l4cs, 0, csum_diff4(rni, 0u, 0u), 0, f.mm);
}

// ipv6_l3: ipv6_dec_hoplimit, then the MACs (smac optional)
__device__ __forceinline__ void frame6_l3(Frame6 &f, const uint32_t *smac, const uint32_t *dmac)
{
    f.hop = (f.hop - 1) & 0xFFu;
    if (smac) { f.smac[0] = smac[0]; f.smac[1] = smac[1]; f.smac_set = true; }
    f.dmac[0] = dmac[0]; f.dmac[1] = dmac[1]; f.dmac_set = true;
}

// ipv6_store_flowlabel(SECLABEL_NB = htonl(identity)): version 6 | the packet's traffic
// class | the label (memory-order word)
__device__ __forceinline__ void frame6_flowlabel(Frame6 &f, uint32_t seclabel)
{
    f.w0 = 0x60u | bswap32(seclabel) | (f.w0 & 0x0000F00Fu);
}

__device__ __forceinline__ void frame6_emit(const Frame6 &f, const uint8_t *in, uint8_t *out, uint32_t stride)
{
    for (uint32_t k = 0; k < stride; k += 16)
        *reinterpret_cast<uint4 *>(out + k) = *reinterpret_cast<const uint4 *>(in + k);
    auto put16 = [&](int off, uint32_t v) { out[off] = (uint8_t)v; out[off + 1] = (uint8_t)(v >> 8); };
    auto put32 = [&](int off, uint32_t v) { put16(off, v & 0xFFFFu); put16(off + 2, v >> 16); };
    if (f.dmac_set) { put32(0, f.dmac[0]); put16(4, f.dmac[1]); }
    if (f.smac_set) { put32(6, f.smac[0]); put16(10, f.smac[1]); }
    put32(14, f.w0);
    out[21] = (uint8_t)f.hop;
#pragma unroll
    for (int j = 0; j < 4; ++j) { put32(22 + 4 * j, f.saddr[j]); put32(38 + 4 * j, f.daddr[j]); }
    if (f.ports) { put16(f.l4off, f.sp); put16(f.l4off + 2, f.dp); }
    if (f.csum) put16(f.l4off + f.coff, f.l4cs);        // after the ports: ICMPv6's field is bytes 2-3
}

// ------------------------------------------------------------------ endpoint ingress programs
// The endpoint program's tables for the IPv4 conntrack stages from its EpHot line
// (one 64-B read); the full EpDev where the event records need its constants or a
// guarded launch needs the CT map's max_entries.
__device__ __forceinline__ EpDev ep_hot4(const DpParams &p, const EpHot &h, uint32_t idx)
{
    EpDev e{};
    e.policy = HashTable{h.pol_buckets, h.pol_vals, h.pol_mask, 32u, (uint32_t)PolicySpec::SPB, h.pol_aux, nullptr, 0};
    e.ct4 = HashTable{h.ct_buckets, h.ct_vals, h.ct_mask, (uint32_t)CT_COLD, (uint32_t)Ct4Spec::SPB, nullptr, h.ct_live,
                      0};
    if (p.ct_guard) e.ct4.cap = G(p.eps)[idx].ct4.cap;
    e.ipv4 = (h.ct_v4 & EPH_V4) ? 1u : 0u;                        // (the stages test LXC_IPV4 for nonzero only)
    e.ct_id = h.ct_v4 & EPH_CT_ID;
    e.seclabel = h.seclabel;
    return e;
}

template <bool FULL>
__device__ __forceinline__ EpDev ep_stage4(const DpParams &p, uint32_t idx)
{
    if constexpr (FULL) return G(p.eps)[idx];
    return ep_hot4(p, G(p.ephot)[idx], idx);
}

// The netdev conntrack stages' view of an endpoint: with one policy and CT4 map for every
// endpoint (p.uni4_on) no per-packet read at all.  Its SECLABEL is then not the
// endpoint's, which only the event records read (those instances take the full entry).
template <bool FULL>
__device__ __forceinline__ EpDev ep_netdev4(const DpParams &p, uint32_t idx)
{
    if constexpr (!FULL)
        if (p.uni4_on && !p.ct_guard) return ep_hot4(p, p.uni4, idx);
    return ep_stage4<FULL>(p, idx);
}

// the same for the IPv6 stages: policy and CT6 tables, SECLABEL
__device__ __forceinline__ EpDev ep_hot6(const DpParams &p, const EpHot &h, uint32_t idx);

template <bool FULL>
__device__ __forceinline__ EpDev ep_stage6(const DpParams &p, uint32_t idx)
{
    if constexpr (FULL) return G(p.eps)[idx];
    return ep_hot6(p, G(p.ephot6)[idx], idx);
}

// ep_netdev4's IPv6 counterpart (one policy and CT6 map for every endpoint: p.uni6_on)
template <bool FULL>
__device__ __forceinline__ EpDev ep_uni6(const DpParams &p, uint32_t idx)
{
    if constexpr (!FULL)
        if (p.uni6_on && !p.ct_guard) return ep_hot6(p, p.uni6, idx);
    return ep_stage6<FULL>(p, idx);
}

__device__ __forceinline__ EpDev ep_hot6(const DpParams &p, const EpHot &h, uint32_t idx)
{
    EpDev e{};
    e.policy = HashTable{h.pol_buckets, h.pol_vals, h.pol_mask, 32u, (uint32_t)PolicySpec::SPB, h.pol_aux, nullptr, 0};
    e.ct6 = HashTable{h.ct_buckets, h.ct_vals, h.ct_mask, (uint32_t)CT_COLD, (uint32_t)Ct6Spec::SPB, nullptr, h.ct_live,
                      0};
    if (p.ct_guard) e.ct6.cap = G(p.eps)[idx].ct6.cap;
    e.seclabel = h.seclabel;
    return e;
}

// After a lane changed conntrack buckets in place (create, delete) on a path that
// reads them with plain loads (FRESH = false): drop this CU's L1 copy, so the lane's
// next lookups see its own change (the atomics that made it bypass L1).
__device__ __forceinline__ void l1_inv() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }

// ipv4_policy (bpf_lxc.c:865-979) + tail_ipv4_policy (:981-993), LXC_NAT46 off.
// Returns the final verdict (TC_ACT_*, drops accounted as METRIC_INGRESS) or E_TRUNC.
// Q: every lane of the wave calls it (live = false: no packet; returns TC_ACT_OK with no
// effect), and the policy lookup is a quad probe at a convergent call site.
template <class M, bool FRESH = true, bool Q = false>
__device__ __forceinline__ int ipv4_policy(const DpParams &p, const EpDev &ep, Skb4 &s, uint32_t src_label,
                                           bool skip_proxy, uint32_t ifindex, uint32_t now, uint8_t &ct_out,
                                           uint16_t &proxy, int32_t &reason, Acct &a, M &m,
                                           RevNatOut *rn = nullptr, bool *defer = nullptr, bool live = true,
                                           uint4 *sq = nullptr)
{
    int ret = 0;
    Tuple4 t{};
    const bool may_defer = defer && *defer;
    if (defer) *defer = false;
    CtState st{0, 0, 0, 0, 0, 0};
    int64_t slot = -1;
    bool mon = false, go = live, dropped = false;
    if (go && s.len < 34) { ret = DROP_INVALID; go = false; dropped = true; }   // revalidate_data
    if (go) {
        t.nexthdr = s.nexthdr;
        t.daddr = s.daddr;
        t.saddr = s.saddr;
        t.dport = t.sport = 0;
        ret = ct_lookup<false, FRESH>(ep.ct4, t, s.h, CT_INGRESS, s.len, now, p.flags, slot, &st, a, &mon);
        if (ret < 0) {
            go = false;
            dropped = true;
        } else {
            ct_out = (uint8_t)ret;
            if (ret == CT_REPLY && st.rev_nat && !st.loopback) {  // lb4_rev_nat(REV_NAT_F_TUPLE_SADDR)
                uint32_t na, np;
                if (revnat4(p, st.rev_nat, na, np, a)) {
                    const int r2 = rev_map_port(s.h, t.nexthdr, np);
                    const int r3 = r2 ? 0 : l4_csum_err(s, t.nexthdr);   // __lb4_rev_nat checksum updates
                    if (r2 || r3) {
                        ret = r2 ? r2 : r3;
                        go = false;
                        dropped = true;
                    } else {
                        t.saddr = na;
                        if (rn) *rn = RevNatOut{true, false, na, np};
                    }
                }
            }
        }
    }
    int verdict = policy_ingress_at<Q>(ep.policy, p.flags, s.len, src_label, t.dport, t.nexthdr, a, go, sq);
    if (go) {
        if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
            if (ret == CT_ESTABLISHED) {
                ct_kill<Ct4Spec>(ep.ct4, slot, a, p.ct_guard);   // ct_delete4
                if (!FRESH) l1_inv();
            }
            ret = DROP_POLICY;
            dropped = true;
        } else {
            if (skip_proxy) verdict = 0;
            if (ret == CT_NEW) {
                if (may_defer) {                                   // k_ct_commit writes it
                    a.nu += 2 * a.ctu;
                    *defer = true;
                } else {
                    CtState sn{0, 0, 0, 0, 0, src_label};
                    const int c = ct_create<false>(ep.ct4, t, s.len, CT_INGRESS, sn, now, a, p.ct_guard, false, true);
                    if (!FRESH) l1_inv();
                    if (is_err(c)) { ret = c; dropped = true; }
                }
            }
            if (!dropped) {
                if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
                    notify_trace(p, m, TRACE_TO_PROXY, s.len, ep.lxc_id, ep.seclabel, 0, 0, HOST_IFINDEX,
                                 (uint32_t)ret, mon);
                    proxy = (uint16_t)verdict;                     // ipv4_redirect_to_host_port
                    return TC_ACT_REDIRECT;                        // redirect(HOST_IFINDEX)
                }
                m.fwd(s.len, METRIC_INGRESS);                      // send_trace_notify(TRACE_TO_LXC)
                notify_trace(p, m, TRACE_TO_LXC, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex,
                             (uint32_t)ret, mon);
                return ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
            }
        }
    }
    if (!dropped) return TC_ACT_OK;                                // (no packet)
    if (ret == E_TRUNC) return ret;
    m.drop(ret, s.len, METRIC_INGRESS);                            // tail_ipv{4,6}_policy: send_drop_notify
    notify_drop(p, m, ret, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex);
    reason = ret;
    return TC_ACT_SHOT;
}

__device__ __forceinline__ bool eq4(const uint32_t *a, const uint32_t *b)
{
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}

// ipv6_policy (bpf_lxc.c:721-849) + tail_ipv6_policy (:851-862); Q / live as ipv4_policy
template <class M, bool FRESH = true, bool Q = false>
__device__ __forceinline__ int ipv6_policy(const DpParams &p, const EpDev &ep, Skb6 &s, uint32_t src_label,
                                           bool skip_proxy, uint32_t ifindex, uint32_t now, uint8_t &ct_out,
                                           uint16_t &proxy, int32_t &reason, Acct &a, M &m,
                                           RevNat6Out *rn = nullptr, bool *defer = nullptr, bool live = true,
                                           uint4 *sq = nullptr)
{
    int ret = 0;
    Tuple6 t{};
    const bool may_defer = defer && *defer;
    if (defer) *defer = false;
    CtState st{0, 0, 0, 0, 0, 0};
    CtState sn{0, 0, 0, 0, 0, src_label};
    int64_t slot = -1;
    bool mon = false, go = live, dropped = false;
    if (go && s.len < 54) { ret = DROP_INVALID; go = false; dropped = true; }
    if (go && s.l4off < 0) { ret = s.l4off; go = false; dropped = true; }   // ipv6_hdrlen error
    if (go) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { t.daddr[j] = s.daddr[j]; t.saddr[j] = s.saddr[j]; }
        t.nexthdr = s.nexthdr;
        t.dport = t.sport = 0;
        sn.rev_nat = s.daddr[3] & 0xFFFFu;                       // derive reverse NAT index (:750-766)
        if (sn.rev_nat && l4_coff6(t.nexthdr)) {                 // zeroed in the packet: L4 checksum
            const int c = l4_csum_err6(s);
            if (c) { ret = c; go = false; dropped = true; }
        }
    }
    if (go) {
        ret = ct_lookup<true, FRESH>(ep.ct6, t, s.h, CT_INGRESS, s.len, now, p.flags, slot, &st, a, &mon);
        if (ret < 0) {
            go = false;
            dropped = true;
        } else {
            ct_out = (uint8_t)ret;
            if (st.rev_nat) {                                    // lb6_rev_nat(.., 0)
                uint32_t na[4], np;
                if (revnat6(p, st.rev_nat, na, np, a)) {
                    const int r2 = rev_map_port(s.h, t.nexthdr, np);
                    const int r3 = r2 ? 0 : l4_csum_err6(s);      // __lb6_rev_nat checksum update
                    if (r2 || r3) {
                        ret = r2 ? r2 : r3;
                        go = false;
                        dropped = true;
                    } else if (rn) {
                        rn->valid = true;
                        rn->np = np;
                        for (int j = 0; j < 4; ++j) rn->na[j] = na[j];
                    }
                }
            }
        }
    }
    int verdict = policy_ingress_at<Q>(ep.policy, p.flags, s.len, src_label, t.dport, t.nexthdr, a, go, sq);
    if (go) {
        if (ret != CT_REPLY && ret != CT_RELATED && verdict < 0) {
            if (ret == CT_ESTABLISHED) {
                ct_kill<Ct6Spec>(ep.ct6, slot, a, p.ct_guard);   // ct_delete6
                if (!FRESH) l1_inv();
            }
            ret = DROP_POLICY;
            dropped = true;
        } else {
            if (skip_proxy) verdict = 0;
            if (ret == CT_NEW) {
                if (may_defer) {
                    a.nu += 2 * a.ctu;
                    *defer = true;
                } else {
                    const int c = ct_create<true>(ep.ct6, t, s.len, CT_INGRESS, sn, now, a, p.ct_guard, false, true);
                    if (!FRESH) l1_inv();
                    if (is_err(c)) { ret = c; dropped = true; }
                }
            }
            if (!dropped) {
                if (verdict > 0 && (ret == CT_NEW || ret == CT_ESTABLISHED)) {
                    notify_trace(p, m, TRACE_TO_PROXY, s.len, ep.lxc_id, ep.seclabel, 0, 0, HOST_IFINDEX,
                                 (uint32_t)ret, mon);
                    proxy = (uint16_t)verdict;
                    return TC_ACT_REDIRECT;
                }
                m.fwd(s.len, METRIC_INGRESS);
                notify_trace(p, m, TRACE_TO_LXC, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex,
                             (uint32_t)ret, mon);
                return ifindex ? TC_ACT_REDIRECT : TC_ACT_OK;
            }
        }
    }
    if (!dropped) return TC_ACT_OK;                                // (no packet)
    if (ret == E_TRUNC) return ret;
    m.drop(ret, s.len, METRIC_INGRESS);                            // tail_ipv{4,6}_policy: send_drop_notify
    notify_drop(p, m, ret, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex);
    reason = ret;
    return TC_ACT_SHOT;
}

// handle_policy (bpf_lxc.c:1003-1038) for an IPv4 / IPv6 packet: DROP_ALL drops
// before any conntrack work; IPv4 needs the endpoint's LXC_IPV4 program.  Q / live as
// ipv4_policy (the policy program's call is convergent: flags are uniform).
template <class M, bool FRESH = true, bool Q = false>
__device__ __forceinline__ int handle_policy4(const DpParams &p, const EpDev &ep, Skb4 &s, uint32_t src_label,
                                              bool skip_proxy, uint32_t ifindex, uint32_t now, uint8_t &ct_out,
                                              uint16_t &proxy, int32_t &reason, Acct &a, M &m,
                                              RevNatOut *rn = nullptr, bool *defer = nullptr, bool live = true,
                                              uint4 *sq = nullptr)
{
    if (defer && ((p.flags & F_DROP_ALL) || !ep.ipv4)) *defer = false;
    const bool run = live && !(p.flags & F_DROP_ALL) && ep.ipv4;
    int r = TC_ACT_OK;
    if (!(p.flags & F_DROP_ALL))
        r = ipv4_policy<M, FRESH, Q>(p, ep, s, src_label, skip_proxy, ifindex, now, ct_out, proxy, reason, a, m, rn,
                                     defer, run, sq);
    if (run || !live) return r;
    const int ret = (p.flags & F_DROP_ALL) ? DROP_POLICY : DROP_UNKNOWN_L3;
    m.drop(ret, s.len, METRIC_INGRESS);                            // bpf_lxc.c:1032-1035
    notify_drop(p, m, ret, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex);
    reason = ret;
    return TC_ACT_SHOT;
}

template <class M, bool FRESH = true, bool Q = false>
__device__ __forceinline__ int handle_policy6(const DpParams &p, const EpDev &ep, Skb6 &s, uint32_t src_label,
                                              bool skip_proxy, uint32_t ifindex, uint32_t now, uint8_t &ct_out,
                                              uint16_t &proxy, int32_t &reason, Acct &a, M &m, RevNat6Out *rn = nullptr,
                                              bool *defer = nullptr, bool live = true, uint4 *sq = nullptr)
{
    if (defer && ((p.flags & F_DROP_ALL) || !ep.ct6.buckets)) *defer = false;
    const bool run = live && !(p.flags & F_DROP_ALL) && ep.ct6.buckets;
    int r = TC_ACT_OK;
    if (!(p.flags & F_DROP_ALL))
        r = ipv6_policy<M, FRESH, Q>(p, ep, s, src_label, skip_proxy, ifindex, now, ct_out, proxy, reason, a, m, rn,
                                     defer, run, sq);
    if (run || !live) return r;
    const int ret = (p.flags & F_DROP_ALL) ? DROP_POLICY : DROP_MISSED_TAIL_CALL;
    m.drop(ret, s.len, METRIC_INGRESS);
    notify_drop(p, m, ret, s.len, ep.lxc_id, src_label, ep.seclabel, ep.lxc_id, ifindex);
    reason = ret;
    return TC_ACT_SHOT;
}

// ------------------------------------------------------------------ grouping
// Packets whose conntrack work can touch a common entry are put in one group and
// run by one lane in packet order; groups are independent, so the batch result
// equals a sequential run on one CPU.  A group is a node of an epoch-tagged open-
// addressing table (hash tag | head of a linked list of packets); the egress path
// also merges nodes with a lock-free union-find (parent pointers per slot).

// find-or-insert the node of 64-bit key hash `gh`; returns its slot
__device__ __forceinline__ uint32_t group_node(const GroupScratch &g, uint64_t gh)
{
    const uint32_t h32 = (uint32_t)gh | 1u;
    const unsigned long long tagged = (unsigned long long)g.epoch << 32 | h32;
    uint32_t s = (uint32_t)(gh >> 32) & g.cap_mask;
    for (;;) {
        unsigned long long cur = __hip_atomic_load(&g.table[2 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == tagged) return s;
        if ((uint32_t)(cur >> 32) != g.epoch) {
            if (__hip_atomic_compare_exchange_strong(&g.table[2 * s], &cur, tagged, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                return s;
            if (cur == tagged) return s;
            if ((uint32_t)(cur >> 32) != g.epoch) continue;
        }
        s = (s + 1) & g.cap_mask;
    }
}

// the node of `gh` if some thread inserted it in this epoch, else NONE
__device__ __forceinline__ uint32_t group_find(const GroupScratch &g, uint64_t gh)
{
    const uint32_t h32 = (uint32_t)gh | 1u;
    const unsigned long long tagged = (unsigned long long)g.epoch << 32 | h32;
    uint32_t s = (uint32_t)(gh >> 32) & g.cap_mask;
    for (uint32_t probes = 0; probes <= g.cap_mask; ++probes) {
        const unsigned long long cur = __hip_atomic_load(&g.table[2 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == tagged) return s;
        if ((uint32_t)(cur >> 32) != g.epoch) return NONE;
        s = (s + 1) & g.cap_mask;
    }
    return NONE;
}

// push packet i on the list of node s; the group's first member (the list tail)
// enters the dense queue q, so the stage that runs the groups has one lane per group
__device__ __forceinline__ void group_push(const GroupScratch &g, uint32_t s, uint32_t i, int q)
{
    const unsigned long long prev = __hip_atomic_exchange(&g.table[2 * s + 1], (unsigned long long)g.epoch << 32 | i,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    g.gslot[i] = s;
    const bool first = (uint32_t)(prev >> 32) != g.epoch;
    g.next[i] = first ? NONE : (uint32_t)prev;
    const uint32_t k = blockIdx.x % QSPLIT;
    const uint32_t at = wave_append(&g.cursor[qctr(q, k)], first);
    if (first) g.queue[((size_t)qbank(q) * QSPLIT + k) * g.qregion + at] = s;
}

// ------------------------------------------------------------------ size-sorted runs
// One lane runs a group's packets one after another, so a wave lasts as long as the
// largest of its 64 groups.  The binned grouping (k_gbin_group, k_heads_place) lists
// the runs {size, members in packet order} of the netdev path in `work` by size class,
// largest first: the groups of one wave then have about the same size.
__host__ __device__ constexpr int size_class(uint32_t n)
{
    return n <= 8 ? (n ? (int)n - 1 : 0) : n <= 12 ? 8 : n <= 16 ? 9 : n <= 24 ? 10 : n <= 32 ? 11
         : n <= 64 ? 12 : n <= 128 ? 13 : n <= 1024 ? 14 : 15;
}

// sub-queue lengths of queue q; returns the number of queued groups
__device__ __forceinline__ uint32_t queue_sizes(const GroupScratch &g, int q, uint32_t *n)
{
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < QSPLIT; ++k) {
        n[k] = __hip_atomic_load(&g.cursor[qctr(q, k)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        total += n[k];
    }
    return total;
}

// the queue word of flat group index j
__device__ __forceinline__ uint32_t *queue_entry(const GroupScratch &g, int q, const uint32_t *n, uint32_t j)
{
    uint32_t k = 0;
#pragma unroll
    for (int t = 0; t < QSPLIT - 1; ++t)
        if (k == (uint32_t)t && j >= n[t]) { j -= n[t]; k = t + 1; }
    return g.queue + ((size_t)qbank(q) * QSPLIT + k) * g.qregion + j;
}

// for every queued group (its slot s and current list head): fn(s, head)
template <class F>
__device__ __forceinline__ void for_each_group(const GroupScratch &g, int q, F &&fn)
{
    uint32_t n[QSPLIT];
    const uint32_t total = queue_sizes(g, q, n);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < total; j += gridDim.x * blockDim.x) {
        const uint32_t s = *queue_entry(g, q, n, j);
        fn(s, (uint32_t)g.table[2 * s + 1]);
    }
}

__device__ __forceinline__ uint32_t uf_parent(const GroupScratch &g, uint32_t s)
{
    const unsigned long long v = __hip_atomic_load(&g.parent[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint32_t)(v >> 32) == g.epoch ? (uint32_t)v : s;
}

__device__ __forceinline__ uint32_t uf_find(const GroupScratch &g, uint32_t s)
{
    for (;;) {
        const uint32_t p = uf_parent(g, s);
        if (p == s) return s;
        const uint32_t gp = uf_parent(g, p);
        if (gp != p) {                                            // path halving (best effort)
            unsigned long long exp = (unsigned long long)g.epoch << 32 | p;
            __hip_atomic_compare_exchange_strong(&g.parent[s], &exp, (unsigned long long)g.epoch << 32 | gp,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s = gp;
    }
}

// merge the groups of nodes a and b: the larger root is linked under the smaller
__device__ __forceinline__ void uf_union(const GroupScratch &g, uint32_t a, uint32_t b)
{
    for (;;) {
        a = uf_find(g, a);
        b = uf_find(g, b);
        if (a == b) return;
        if (a < b) { const uint32_t x = a; a = b; b = x; }
        unsigned long long cur = __hip_atomic_load(&g.parent[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(cur >> 32) == g.epoch && (uint32_t)cur != a) continue;   // no longer a root
        if (__hip_atomic_compare_exchange_strong(&g.parent[a], &cur, (unsigned long long)g.epoch << 32 | b,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

// The walkers trust no list word: a packet index past the launch, or a run {size, members}
// reaching past `order`'s 2 * lim words (a stale or corrupt list), is stored in g.err --
// host-mapped, so the context fails its next call with -EPROTO without a device wait --
// and skipped, never dereferenced.
__device__ __noinline__ void group_err(const GroupScratch &g, uint32_t code)
{
    if (g.err) __hip_atomic_store(g.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool pkt_ok(const GroupScratch &g, uint32_t x)
{
    if (x < g.lim) return true;
    group_err(g, GERR_INDEX);
    return false;
}
// the run at `off` with `cnt` members fits `order` (1 + cnt words from off)
__device__ __forceinline__ bool run_ok(const GroupScratch &g, uint32_t off, uint32_t cnt)
{
    const uint32_t words = 2u * g.lim;
    if (off < words && cnt >= 1u && cnt < words - off) return true;
    group_err(g, GERR_INDEX);
    return false;
}

// fn(i, run size) for every member of every listed run of queue q, runs in `work`
// order and members in packet order, then every singleton group (listed densely in
// `single`); the next member's index is loaded while fn runs.
template <class F>
__device__ __forceinline__ void for_each_run(const GroupScratch &g, int q, bool first_only, F &&fn, uint32_t skip = 0)
{
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    auto run = [&](uint32_t off) {
        if (off >= 2u * g.lim) { group_err(g, GERR_INDEX); return; }
        const uint32_t cnt = first_only ? 1u : g.order[off];
        if (!run_ok(g, off, cnt)) return;
        uint32_t v = g.order[off + 1];
#pragma unroll 1
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint32_t vn = k + 1 < cnt ? g.order[off + 2 + k] : NONE;
            if (pkt_ok(g, v)) fn(v, cnt);
            v = vn;
        }
    };
    uint32_t multi = 0;                                           // listed runs: classes >= 1
#pragma unroll
    for (int c = 1; c < NCLASS; ++c) multi += g.cursor[qcls(q, c)];
    for (uint32_t j = skip + tid; j < multi; j += stride) run(g.work[j]);   // (skip: the hot runs, k_ct_hot)
    const uint32_t singles = g.cursor[SINGLE_WORD0 + q];
    for (uint32_t j = tid; j < singles; j += stride) {
        const uint32_t x = g.single[j];
        if (pkt_ok(g, x)) fn(x, 1u);
    }
}

// fn(i) for member `pos` of every group of queue q (position lists, g.flat), in packet
// order; the last lists (pos = NPOS - 1 .. 15, by size class) name runs: fn for their
// members from pos on.
// One call site of fn.
template <class F>
__device__ __forceinline__ void for_each_at(const GroupScratch &g, int q, uint32_t pos, F &&fn)
{
    uint32_t base = 0;
    for (uint32_t l = 0; l < pos; ++l) base += g.cursor[qcls(q, l)];
    const bool runs = pos + 1 == NPOS;
    uint32_t total = g.cursor[qcls(q, pos)];
    if (runs)                                                     // (the continuation: lists pos .. 15, one
        for (uint32_t l = pos + 1; l < 16; ++l) total += g.cursor[qcls(q, l)];   //  per size class, in order)
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
    for (uint32_t j = tid; j < total; j += stride) {
        const uint32_t e = g.work[base + j];
        uint32_t k1 = pos + 1;
        if (runs) {
            if (e >= 2u * g.lim) { group_err(g, GERR_INDEX); continue; }
            k1 = g.order[e];
            if (!run_ok(g, e, k1)) continue;
        }
#pragma unroll 1
        for (uint32_t k = pos; k < k1; ++k) {
            const uint32_t x = runs ? g.order[e + 1 + k] : e;
            if (pkt_ok(g, x)) fn(x);
        }
    }
}

// node key of an unordered address pair (v4 words or v6 4-word addresses), mixed
// with a salt that separates families / stages
__device__ __forceinline__ uint64_t pair_hash4(uint32_t a, uint32_t b, uint64_t salt)
{
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    return mix64(((uint64_t)lo << 32 | hi) ^ salt);
}

__device__ __forceinline__ bool lt6(const uint32_t *a, const uint32_t *b)
{
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (a[j] != b[j]) return a[j] < b[j];
    return false;
}

__device__ __forceinline__ uint64_t pair_hash6(const uint32_t *a, const uint32_t *b, uint64_t salt)
{
    const uint32_t *lo = lt6(a, b) ? a : b, *hi = lt6(a, b) ? b : a;
    uint64_t h = salt ^ 0x6A09E667F3BCC908ULL;
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
        h = mix64(h ^ ((uint64_t)lo[j] | (uint64_t)lo[j + 1] << 32)) + 0x9E3779B97F4A7C15ULL;
        h = mix64(h ^ ((uint64_t)hi[j] | (uint64_t)hi[j + 1] << 32)) + 0x9E3779B97F4A7C15ULL;
    }
    return mix64(h);
}

}  // namespace cv
