// cv_hash.hpp — device-resident exact-match tables (the HASH / LRU_HASH maps of the
// reference: cilium_lxc, v4_fix/v6_fix, cilium_policy_*, cilium_ct4_*, lb services).
//
// Layout, sized for HBM3E lines: a table is nb (power of two) buckets of BW 32-bit
// words (64 or 128 B, one cache line).  Word 0-1 hold one tag byte per slot
// (0 empty, 1 dead, 2 busy, 3..255 hash fingerprint); then SPB keys of KW words;
// then SPB inline values of IVW words, or of one 16-bit halfword each (IVH = 1, the
// policy table's proxy_port).  Larger values live in a side array indexed
// by slot (bucket * SPB + slot) with a fixed byte stride.  Conntrack buckets (KS >
// KW) interleave each slot's key with the hot words of its entry (cv_dev.hpp
// ct_hot), so a hit reads one line.  Tag 2 marks a slot a
// device thread is claiming (skipped by lookups, never matched).  Linear probing over
// buckets; a lookup ends at the first bucket holding an empty slot, so one probe
// is one line read in the common case.  The same code runs on the host (table
// build) and on the device (lookups, conntrack inserts).
#pragma once
#include "cv_common.hpp"

namespace cv {

constexpr uint32_t TAG_EMPTY = 0, TAG_DEAD = 1, TAG_BUSY = 2;
constexpr int MAX_PROBE = 64;        // probe limit (buckets) of the host-built tables: a longer chain grows the table
// Conntrack tables (filled on the device, never rebuilt) probe up to CT_MAX_PROBE
// buckets: a create fails below max_entries only when that many consecutive buckets
// hold live entries and nothing else.  The tables are sized for max_entries at 60 %
// slot load (buckets_for), where a run of k full 2-slot buckets has probability about
// e^(-0.22 k): e^-900 for k = 4096, so a create below max_entries never fails -- the
// kernel hash map's behaviour -- while a lookup miss still ends at the first bucket
// with an empty slot (k_ct_gc turns tombstones back into empty slots).
constexpr int CT_MAX_PROBE = 4096;
constexpr uint64_t HASH_SEED = 0x243F6A8885A308D3ULL;

struct HashTable {            // POD view, passed by value to kernels
    uint32_t *buckets;        // nb * BW words
    uint8_t  *vals;           // nb * SPB * vstride bytes, or null
    uint64_t  mask;           // nb - 1
    uint32_t  vstride;
    uint32_t  spb;
    unsigned long long *aux;  // per-slot 64-bit side words (policy counter deltas), or null
    unsigned long long *live; // conntrack maps: the live-entry count (device), or null
    uint64_t  cap;            // conntrack maps: max_entries (a create past it fails, -E2BIG)
};

template <int KW_, int IVW_, int SPB_, int BW_, int IVH_ = 0, int SYM_ = 0, int KS_ = 0>
struct HashSpec {
    static constexpr int KW = KW_, IVW = IVW_, SPB = SPB_, BW = BW_, IVH = IVH_, SYM = SYM_;
    static constexpr int KS = KS_ ? KS_ : KW_;                   // words from one slot's key to the next
    static constexpr int KEY0 = 2, IVAL0 = 2 + SPB * KS, HVAL0 = 2 * IVAL0;   // HVAL0 in halfwords
    static constexpr int MAXP = SYM ? CT_MAX_PROBE : MAX_PROBE;           // probe limit in buckets
    static_assert(IVAL0 + SPB * IVW <= BW, "bucket overflow");
    static_assert(IVH == 0 || (IVW == 0 && IVH == 1 && HVAL0 + SPB <= 2 * BW), "halfword values");
    static_assert(SPB <= 8, "eight tag bytes");
    static_assert(BW % 4 == 0, "bucket = whole 16-B vectors");
};

// table shapes per role
using LxcV4Spec  = HashSpec<1, 1, 7, 16>;   // ip4 -> {lxc_id | HOST<<16 | ifindex!=0 <<17}
using LxcV6Spec  = HashSpec<4, 1, 6, 32>;
using Cidr4Spec  = HashSpec<1, 0, 8, 16>;   // /32 deny set (v4_fix)
using Cidr6Spec  = HashSpec<4, 0, 7, 32>;   // /128 deny set (v6_fix)
using PolicySpec = HashSpec<2, 0, 5, 16, 1>; // policy_key (8 B) -> inline proxy_port; side array policy_entry (stride 32)
// conntrack: {key, 10 hot words of struct ct_entry} per slot, the rest in 32-B side slots
using Ct4Spec    = HashSpec<4, 0, 2, 32, 0, 1, 14>;   // ipv4_ct_tuple (14 B + 2 zero): 2 slots per 128 B
using Ct6Spec    = HashSpec<10, 0, 3, 64, 0, 1, 20>;  // ipv6_ct_tuple (40 B): 3 slots per 256 B
constexpr int CT_HOTW = 10, CT_COLD = 32;   // hot words per CT slot; bytes per CT side slot
using Lb4Spec    = HashSpec<2, 3, 6, 32>;   // lb4_key (8 B) -> lb4_service (12 B) inline
using Lb6Spec    = HashSpec<5, 6, 4, 64>;   // lb6_key (20 B) -> lb6_service (24 B) inline
using Lpm6Spec   = HashSpec<5, 1, 5, 32>;   // (masked v6 addr, plen) -> value

CV_HD uint32_t tag_of(uint64_t h)
{
    uint32_t t = (uint32_t)(h >> 56);
    return t < 3 ? t + 3 : t;
}

template <class S>
CV_HD uint32_t half_at(const uint32_t *w, int h) { return (w[h >> 1] >> (16 * (h & 1))) & 0xFFFFu; }

template <class S>
CV_HD uint64_t key_hash(const uint32_t *key) { return hash_words<S::KW>(key, HASH_SEED); }

// The home-bucket hash of a key and its fingerprint.  Conntrack tables (SYM) place a
// tuple by its direction-free form -- the (address, port) endpoints in sorted order,
// TUPLE_F_IN cleared -- so a tuple and its reverse (the two keys ct_lookup4/6 try,
// conntrack.h:442-562 / 286-412) share a home bucket and one bucket read answers
// both; the fingerprint comes from the full key and still tells them apart.
template <class S>
CV_HD uint64_t home_hash(const uint32_t *key, uint32_t &tag)
{
    const uint64_t h = key_hash<S>(key);
    tag = tag_of(h);
    if constexpr (S::SYM != 0) {
        constexpr int A = S::KW == 4 ? 1 : 4;                    // words per address
        const uint32_t *da = key, *sa = key + A;
        const uint32_t ports = key[2 * A], dp = ports & 0xFFFFu, sp = ports >> 16;
        bool d_lt = dp < sp;                                     // order the (address, port) endpoints
#pragma unroll
        for (int j = A - 1; j >= 0; --j)
            if (da[j] != sa[j]) d_lt = da[j] < sa[j];
        uint32_t sym[S::KW];
#pragma unroll
        for (int j = 0; j < A; ++j) { sym[j] = d_lt ? da[j] : sa[j]; sym[A + j] = d_lt ? sa[j] : da[j]; }
        sym[2 * A] = d_lt ? (dp | sp << 16) : (sp | dp << 16);
        sym[2 * A + 1] = key[2 * A + 1] & ~((uint32_t)TUPLE_F_IN << 8);
        return hash_words<S::KW>(sym, HASH_SEED ^ 0x5CA1AB1E0DDBA11ULL);
    }
    return h;
}

// Match `key` in one bucket snapshot w[BW].  Returns the slot or -1; *stop is set
// when the bucket has an empty slot (end of the probe chain).
template <class S>
CV_HD int match_bucket(const uint32_t *w, const uint32_t *key, uint32_t tag, bool *stop)
{
    uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    int hit = -1;
    bool empty = false;
#pragma unroll
    for (int s = S::SPB - 1; s >= 0; --s) {
        uint32_t t = (uint32_t)(tags >> (8 * s)) & 0xFFu;
        empty |= (t == TAG_EMPTY);
        bool eq = (t == tag);
#pragma unroll
        for (int j = 0; j < S::KW; ++j) eq &= (w[S::KEY0 + s * S::KS + j] == key[j]);
        hit = eq ? s : hit;
    }
    *stop = empty;
    return hit;
}

// ---------------------------------------------------------------- device lookup
// Bucket words of a table the launch also writes (conntrack, S::SYM) are read past
// the CU's L1 (agent-scope loads, served by the XCD's L2) where FRESH: a lane's own
// claims and kills are atomics, which drop the line from its L2 but not necessarily
// from its L1, so a plain re-read of a bucket it just changed could return the old
// tags or key.  Callers that invalidate their L1 after their own (rare) bucket
// changes read with plain loads instead (FRESH = false): the tags and the key then
// come from one L1 line fill.
template <class S, bool FRESH = true>
__device__ __forceinline__ uint2 ld_tags(const CV_G uint32_t *bw)
{
    if constexpr (S::SYM != 0 && FRESH) {
        const unsigned long long v = __hip_atomic_load(reinterpret_cast<const CV_G unsigned long long *>(bw),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    }
    return *reinterpret_cast<const CV_G uint2 *>(bw);
}

// the stored key at kw equals key (kw is 8-B aligned: KEY0 = 2 and even KW for SYM specs)
template <class S, bool FRESH = true>
__device__ __forceinline__ bool key_eq(const CV_G uint32_t *kw, const uint32_t *key)
{
    bool eq = true;
    if constexpr (S::SYM != 0 && FRESH) {
        static_assert(S::KW % 2 == 0 && S::KEY0 % 2 == 0, "8-B key words");
#pragma unroll
        for (int j = 0; j < S::KW; j += 2) {
            const unsigned long long v = __hip_atomic_load(reinterpret_cast<const CV_G unsigned long long *>(kw + j),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            eq &= ((uint32_t)v == key[j]) & ((uint32_t)(v >> 32) == key[j + 1]);
        }
    } else if constexpr (S::SYM != 0) {
#pragma unroll
        for (int j = 0; j < S::KW; j += 2) {
            const uint2 v = *reinterpret_cast<const CV_G uint2 *>(kw + j);
            eq &= (v.x == key[j]) & (v.y == key[j + 1]);
        }
    } else if constexpr (S::KW % 2 == 0 && S::KEY0 % 2 == 0 && S::KS % 2 == 0) {
        // 8-B aligned key words (buckets are 64-B aligned): half the load instructions
#pragma unroll
        for (int j = 0; j < S::KW; j += 2) {
            const uint2 v = *reinterpret_cast<const CV_G uint2 *>(kw + j);
            eq &= (v.x == key[j]) & (v.y == key[j + 1]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < S::KW; ++j) eq &= (kw[j] == key[j]);
    }
    return eq;
}

// the inline value words of slot sl of a bucket (wide loads where the words are 8-B
// aligned, a 12-B load for the lb4_service triple)
template <class S>
__device__ __forceinline__ void ival_load(const CV_G uint32_t *bw, int sl, uint32_t *ival)
{
    const CV_G uint32_t *iv = bw + S::IVAL0 + sl * S::IVW;
    if constexpr (S::IVW == 3) {
        const uint3 v = *reinterpret_cast<const CV_G uint3 *>(iv);
        ival[0] = v.x; ival[1] = v.y; ival[2] = v.z;
    } else if constexpr (S::IVW % 2 == 0 && S::IVAL0 % 2 == 0) {
#pragma unroll
        for (int j = 0; j < S::IVW; j += 2) {
            const uint2 v = *reinterpret_cast<const CV_G uint2 *>(iv + j);
            ival[j] = v.x; ival[j + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < S::IVW; ++j) ival[j] = iv[j];
    }
}
template <class S>
__device__ __forceinline__ void load_bucket(const uint32_t *__restrict__ buckets, uint64_t b, uint32_t (&w)[S::BW])
{
    const CV_G uint4 *q = reinterpret_cast<const CV_G uint4 *>(G(buckets) + b * S::BW);
#pragma unroll
    for (int i = 0; i < S::BW / 4; ++i) {
        uint4 v = q[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
}

// bytes of the 8 tag bytes equal to `tag` (bit 7 of each matching byte), and empty slots
template <class S>
__device__ __forceinline__ void tag_masks(uint64_t tags, uint32_t tag, uint64_t &match, bool &empty)
{
    constexpr uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
    constexpr uint64_t valid = S::SPB >= 8 ? ~0ULL : ((1ULL << (8 * S::SPB)) - 1);
    const uint64_t x = tags ^ (ones * tag);
    match = (x - ones) & ~x & highs & valid;                       // zero bytes of x (exact for tag >= 3)
    const uint64_t e = (tags - ones) & ~tags & highs & valid;       // zero bytes of tags: empty slots
    empty = e != 0;
}

// Tag-first probe for wide buckets (>= 128 B): read the 8 tag bytes, then only the
// keys (and inline values) of slots whose fingerprint matches, so a probe keeps a
// few registers live instead of the whole bucket.  Same result as the full-bucket
// match: a key is stored once; the chain ends at a bucket with an empty slot.
template <class S, bool FRESH = true>
__device__ __forceinline__ int64_t dev_find_tf(const HashTable &t, const uint32_t *key, uint32_t *ival)
{
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    uint64_t b = h & t.mask;
    for (int p = 0; p < S::MAXP; ++p) {
        const CV_G uint32_t *bw = G(t.buckets) + b * S::BW;
        const uint2 tg = ld_tags<S, FRESH>(bw);
        uint64_t match;
        bool empty;
        tag_masks<S>((uint64_t)tg.x | ((uint64_t)tg.y << 32), tag, match, empty);
        while (match) {
            const int sl = (__builtin_ctzll(match) >> 3);
            match &= match - 1;
            const CV_G uint32_t *kw = bw + S::KEY0 + sl * S::KS;
            const bool eq = key_eq<S, FRESH>(kw, key);
            if (eq) {
                ival_load<S>(bw, sl, ival);
                if (S::IVH) ival[0] = half_at<S>(bw, S::HVAL0 + sl);
                return (int64_t)(b * S::SPB + sl);
            }
        }
        if (empty) return -1;
        b = (b + 1) & t.mask;
    }
    return -1;
}

// the full-bucket probe chain from bucket b (probe number p0 of S::MAXP)
template <class S>
__device__ __forceinline__ int64_t dev_find_from(const HashTable &t, const uint32_t *key, uint32_t tag, uint64_t b,
                                                 int p0, uint32_t *ival);

// Returns the slot index (bucket * SPB + slot) or -1; copies the inline value.
template <class S, bool FRESH = true>
__device__ __forceinline__ int64_t dev_find(const HashTable &t, const uint32_t *key, uint32_t *ival)
{
    if (!t.buckets) return -1;
    if constexpr (S::BW >= 32) return dev_find_tf<S, FRESH>(t, key, ival);   // (tag-first 64-B probes: slower)
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    return dev_find_from<S>(t, key, tag, h & t.mask, 0, ival);
}

template <class S>
__device__ __forceinline__ int64_t dev_find_from(const HashTable &t, const uint32_t *key, uint32_t tag, uint64_t b,
                                                 int p0, uint32_t *ival)
{
    for (int p = p0; p < S::MAXP; ++p) {
        uint32_t w[S::BW];
        load_bucket<S>(t.buckets, b, w);
        bool stop;
        int s = match_bucket<S>(w, key, tag, &stop);
        if (s >= 0) {
#pragma unroll
            for (int q = 0; q < S::SPB; ++q) {     // select without a runtime register index
#pragma unroll
                for (int j = 0; j < S::IVW; ++j)
                    if (q == s) ival[j] = w[S::IVAL0 + q * S::IVW + j];
                if (S::IVH && q == s) ival[0] = half_at<S>(w, S::HVAL0 + q);
            }
            return (int64_t)(b * S::SPB + s);
        }
        if (stop) return -1;
        b = (b + 1) & t.mask;
    }
    return -1;
}

// ---------------------------------------------------------------- split-phase probe
// ---------------------------------------------------------------- quad probes
// A lane reading a whole 64-B bucket alone issues four 16-B loads to one line: four
// line accesses in the texture path for 64 bytes.  Here the 4 lanes of a quad read
// each other's home buckets together: in round k every lane of the quad loads one
// 16-B part of quad-lane k's bucket, straight into LDS (global_load_lds_dwordx4), so
// one wave-instruction touches 16 lines instead of 64; each lane then reads its own
// bucket back from LDS.  Round k's lane r loads part (r + k) & 3, which places the 4
// parts a lane reads back for one part index in 4 different LDS banks.
//
// Every lane of the wave must call it at the same point (quad-lane broadcasts);
// `mine` = the lane's bucket or null (no lookup).  `st`: the wave's 4 KiB LDS stage.
template <int K>
__device__ __forceinline__ void quad_round(int plo, int phi, int r, uint4 *st)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp(plo, K * 0x55, 0xF, 0xF, false);   // quad_perm [K,K,K,K]
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp(phi, K * 0x55, 0xF, 0xF, false);
    const uint32_t *src = reinterpret_cast<const uint32_t *>((uintptr_t)((uint64_t)hi << 32 | lo));
    if (src) __builtin_amdgcn_global_load_lds(src + 4 * ((r + K) & 3), st + K * 64, 16, 0, 0);
}

__device__ __forceinline__ void quad_load64(const uint32_t *mine, uint4 *st, uint32_t (&w)[16])
{
    const int lane = (int)(threadIdx.x & 63), r = lane & 3, qb = lane & ~3;
    const uint64_t pm = (uint64_t)(uintptr_t)mine;
    const int plo = (int)(uint32_t)pm, phi = (int)(uint32_t)(pm >> 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");            // earlier LDS reads of st are done
    __builtin_amdgcn_wave_barrier();
    quad_round<0>(plo, phi, r, st);
    quad_round<1>(plo, phi, r, st);
    quad_round<2>(plo, phi, r, st);
    quad_round<3>(plo, phi, r, st);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (mine) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 v = st[r * 64 + qb + ((j - r) & 3)];
            w[4 * j] = v.x; w[4 * j + 1] = v.y; w[4 * j + 2] = v.z; w[4 * j + 3] = v.w;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// two buckets per lane in one pass (8 rounds, one wait): stage `st` holds 8 KiB
__device__ __forceinline__ void quad_load64x2(const uint32_t *m0, const uint32_t *m1, uint4 *st, uint32_t (&w0)[16],
                                              uint32_t (&w1)[16])
{
    const int lane = (int)(threadIdx.x & 63), r = lane & 3, qb = lane & ~3;
    const uint64_t p0 = (uint64_t)(uintptr_t)m0, p1 = (uint64_t)(uintptr_t)m1;
    const int lo0 = (int)(uint32_t)p0, hi0 = (int)(uint32_t)(p0 >> 32);
    const int lo1 = (int)(uint32_t)p1, hi1 = (int)(uint32_t)(p1 >> 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    quad_round<0>(lo0, hi0, r, st);
    quad_round<1>(lo0, hi0, r, st);
    quad_round<2>(lo0, hi0, r, st);
    quad_round<3>(lo0, hi0, r, st);
    quad_round<0>(lo1, hi1, r, st + 256);
    quad_round<1>(lo1, hi1, r, st + 256);
    quad_round<2>(lo1, hi1, r, st + 256);
    quad_round<3>(lo1, hi1, r, st + 256);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (m0) {
            const uint4 v = st[r * 64 + qb + ((j - r) & 3)];
            w0[4 * j] = v.x; w0[4 * j + 1] = v.y; w0[4 * j + 2] = v.z; w0[4 * j + 3] = v.w;
        }
        if (m1) {
            const uint4 v = st[256 + r * 64 + qb + ((j - r) & 3)];
            w1[4 * j] = v.x; w1[4 * j + 1] = v.y; w1[4 * j + 2] = v.z; w1[4 * j + 3] = v.w;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// the bucket snapshot w of bucket b: slot index or -1 (chain continued lane by lane)
template <class S>
__device__ __forceinline__ int64_t quad_match(const HashTable &t, const uint32_t *key, uint32_t tag, uint64_t b,
                                              const uint32_t (&w)[16], uint32_t *ival)
{
    bool stop;
    const int s = match_bucket<S>(w, key, tag, &stop);
    if (s >= 0) {
#pragma unroll
        for (int q = 0; q < S::SPB; ++q) {
#pragma unroll
            for (int j = 0; j < S::IVW; ++j)
                if (q == s) ival[j] = w[S::IVAL0 + q * S::IVW + j];
            if (S::IVH && q == s) ival[0] = half_at<S>(w, S::HVAL0 + q);
        }
        return (int64_t)(b * S::SPB + s);
    }
    if (stop) return -1;
    return dev_find_from<S>(t, key, tag, (b + 1) & t.mask, 1, ival);
}

// two quad_find in one pass
template <class S>
__device__ __forceinline__ void quad_find2(const HashTable &t, const uint32_t *k0, bool want0, const uint32_t *k1,
                                           bool want1, uint4 *st, int64_t &s0, uint32_t *iv0, int64_t &s1,
                                           uint32_t *iv1)
{
    uint32_t tg0, tg1;
    const uint64_t h0 = home_hash<S>(k0, tg0), h1 = home_hash<S>(k1, tg1);
    const uint64_t b0 = h0 & t.mask, b1 = h1 & t.mask;
    const uint32_t *bw0 = (want0 && t.buckets) ? t.buckets + b0 * S::BW : nullptr;
    const uint32_t *bw1 = (want1 && t.buckets) ? t.buckets + b1 * S::BW : nullptr;
    uint32_t w0[16], w1[16];
    quad_load64x2(bw0, bw1, st, w0, w1);
    s0 = bw0 ? quad_match<S>(t, k0, tg0, b0, w0, iv0) : -1;
    s1 = bw1 ? quad_match<S>(t, k1, tg1, b1, w1, iv1) : -1;
}

// dev_find for 64-B buckets through quad_load64 (same result); `want` false: no
// lookup (the lane still takes part)
template <class S>
__device__ __forceinline__ int64_t quad_find(const HashTable &t, const uint32_t *key, bool want, uint4 *st,
                                             uint32_t *ival)
{
    static_assert(S::BW == 16, "64-B buckets");
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    const uint64_t b = h & t.mask;
    const uint32_t *bw = (want && t.buckets) ? t.buckets + b * S::BW : nullptr;
    if (!__ballot(bw != nullptr)) return -1;                      // (wave-uniform: no lane looks up)
    uint32_t w[16];
    quad_load64(bw, st, w);
    if (!bw) return -1;
    bool stop;
    const int s = match_bucket<S>(w, key, tag, &stop);
    if (s >= 0) {
#pragma unroll
        for (int q = 0; q < S::SPB; ++q) {
#pragma unroll
            for (int j = 0; j < S::IVW; ++j)
                if (q == s) ival[j] = w[S::IVAL0 + q * S::IVW + j];
            if (S::IVH && q == s) ival[0] = half_at<S>(w, S::HVAL0 + q);
        }
        return (int64_t)(b * S::SPB + s);
    }
    if (stop) return -1;
    return dev_find_from<S>(t, key, tag, (b + 1) & t.mask, 1, ival);   // rare: the chain goes on
}

// probe_begin issues the home bucket's first load (tags for wide buckets, the whole
// 64-B line for narrow ones) and returns at once; probe_end waits for it and
// finishes the lookup (following the probe chain when the home bucket is full).
// Beginning several independent lookups before ending any keeps their first memory
// round trips in flight together: a dependent-latency chain becomes one round trip.
template <class S>
struct Probe {
    const CV_G uint32_t *bw;
    uint64_t b;
    uint32_t tag;
    uint32_t w[S::BW >= 32 ? 2 : S::BW];
};

template <class S, bool FRESH = true>
__device__ __forceinline__ Probe<S> probe_begin(const HashTable &t, const uint32_t *key)
{
    Probe<S> pr;
    const uint64_t h = home_hash<S>(key, pr.tag);
    pr.b = h & t.mask;
    pr.bw = t.buckets ? G(t.buckets) + pr.b * S::BW : nullptr;
    if (!pr.bw) return pr;
    if constexpr (S::BW >= 32) {
        const uint2 tg = ld_tags<S, FRESH>(pr.bw);
        pr.w[0] = tg.x; pr.w[1] = tg.y;
    } else {
        const CV_G uint4 *q = reinterpret_cast<const CV_G uint4 *>(pr.bw);
#pragma unroll
        for (int i = 0; i < S::BW / 4; ++i) {
            const uint4 v = q[i];
            pr.w[4 * i] = v.x; pr.w[4 * i + 1] = v.y; pr.w[4 * i + 2] = v.z; pr.w[4 * i + 3] = v.w;
        }
    }
    return pr;
}

template <class S, bool FRESH = true>
__device__ __forceinline__ int64_t probe_end(const Probe<S> &pr, const HashTable &t, const uint32_t *key, uint32_t *ival)
{
    if (!pr.bw) return -1;
    uint64_t b = pr.b;
    bool stop;
    if constexpr (S::BW >= 32) {
        uint64_t match;
        tag_masks<S>((uint64_t)pr.w[0] | ((uint64_t)pr.w[1] << 32), pr.tag, match, stop);
        while (match) {
            const int sl = (__builtin_ctzll(match) >> 3);
            match &= match - 1;
            const CV_G uint32_t *kw = pr.bw + S::KEY0 + sl * S::KS;
            const bool eq = key_eq<S, FRESH>(kw, key);
            if (eq) {
                ival_load<S>(pr.bw, sl, ival);
                return (int64_t)(b * S::SPB + sl);
            }
        }
    } else {
        const int s = match_bucket<S>(pr.w, key, pr.tag, &stop);
        if (s >= 0) {
#pragma unroll
            for (int q = 0; q < S::SPB; ++q) {
#pragma unroll
                for (int j = 0; j < S::IVW; ++j)
                    if (q == s) ival[j] = pr.w[S::IVAL0 + q * S::IVW + j];
                if (S::IVH && q == s) ival[0] = half_at<S>(pr.w, S::HVAL0 + q);
            }
            return (int64_t)(b * S::SPB + s);
        }
    }
    if (stop) return -1;
    // rare: the home bucket is full, continue the chain from the next bucket
    for (int p = 1; p < S::MAXP; ++p) {
        b = (b + 1) & t.mask;
        Probe<S> nx;
        nx.tag = pr.tag;
        nx.b = b;
        nx.bw = G(t.buckets) + b * S::BW;
        if constexpr (S::BW >= 32) {
            const uint2 tg = ld_tags<S, FRESH>(nx.bw);
            uint64_t match;
            tag_masks<S>((uint64_t)tg.x | ((uint64_t)tg.y << 32), pr.tag, match, stop);
            while (match) {
                const int sl = (__builtin_ctzll(match) >> 3);
                match &= match - 1;
                const CV_G uint32_t *kw = nx.bw + S::KEY0 + sl * S::KS;
                const bool eq = key_eq<S, FRESH>(kw, key);
                if (eq) {
                    ival_load<S>(nx.bw, sl, ival);
                    return (int64_t)(b * S::SPB + sl);
                }
            }
        } else {
            uint32_t w[S::BW];
            load_bucket<S>(t.buckets, b, w);
            const int s = match_bucket<S>(w, key, pr.tag, &stop);
            if (s >= 0) {
#pragma unroll
                for (int q = 0; q < S::SPB; ++q) {
#pragma unroll
                    for (int j = 0; j < S::IVW; ++j)
                        if (q == s) ival[j] = w[S::IVAL0 + q * S::IVW + j];
                    if (S::IVH && q == s) ival[0] = half_at<S>(w, S::HVAL0 + q);
                }
                return (int64_t)(b * S::SPB + s);
            }
        }
        if (stop) return -1;
    }
    return -1;
}

// Conntrack insert (map_update_elem BPF_ANY on an LRU_HASH, conntrack.h:694,720,740).
// The caller guarantees that no other thread of the launch touches `key` (packets
// are grouped by address pair), so the only race is for free slots.  One pass over
// the probe chain finds the key or, failing that, the first bucket with a free
// (empty / dead) slot; the slot is claimed by ONE agent-scope CAS of its tag word
// that writes the fingerprint (the snapshot the pass read is the CAS's first
// guess; a lost race returns the current word and the claim moves on), then the key
// is written.  Returns the slot, or -1 when the probe limit is hit
// (-> DROP_CT_CREATE_FAILED); *created tells whether the key was new.
// known_absent: the caller's lookup of `key` missed in this launch (a create right
// after ct_lookup), so no key compare is needed and the first free slot is taken.
// No fence between the fingerprint and the key (an agent-scope release is a
// write-back of the whole XCD L2, microseconds per create): the only thread that
// looks `key` up in this launch is this one (program order), and any other reader
// whose fingerprint collides sees either the new key or the zero words every free
// slot holds (dev_kill and the GC clear a key before its slot turns dead), neither of
// which is its own key.  The kernel boundary publishes the entry to later launches.
__device__ __forceinline__ bool claim_in_word(CV_G uint32_t *tw, uint32_t cur, int first, int nslots, uint32_t tag,
                                              int &got, uint32_t &was)
{
    for (;;) {
        int k = -1;
#pragma unroll
        for (int q = 3; q >= 0; --q)
            if (q < nslots && ((cur >> (8 * q)) & 0xFFu) < TAG_BUSY) k = q;
        if (k < 0) return false;
        const uint32_t nw = (cur & ~(0xFFu << (8 * k))) | (tag << (8 * k));
        const uint32_t old = (cur >> (8 * k)) & 0xFFu;
        if (__hip_atomic_compare_exchange_strong(tw, &cur, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            got = first + k;
            was = old;
            return true;
        }
    }
}

template <class S>
__device__ __forceinline__ int64_t dev_upsert(const HashTable &t, const uint32_t *key, bool *created,
                                              bool known_absent = false, uint32_t *was = nullptr)
{
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    constexpr uint64_t valid = S::SPB >= 8 ? ~0ULL : ((1ULL << (8 * S::SPB)) - 1);
    constexpr uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
    *created = false;
    uint64_t b = h & t.mask, fb = 0;
    uint64_t ftags = 0;
    bool have_free = false;
    for (int p = 0; p < S::MAXP; ++p) {                          // 1) the key, and the first free slot
        const CV_G uint32_t *bw = G(t.buckets) + b * S::BW;
        const uint2 tg = ld_tags<S>(bw);
        const uint64_t tags = (uint64_t)tg.x | ((uint64_t)tg.y << 32);
        uint64_t match;
        bool empty;
        tag_masks<S>(tags, tag, match, empty);
        while (!known_absent && match) {
            const int sl = (__builtin_ctzll(match) >> 3);
            match &= match - 1;
            const CV_G uint32_t *kw = bw + S::KEY0 + sl * S::KS;
            const bool eq = key_eq<S>(kw, key);
            if (eq) return (int64_t)(b * S::SPB + sl);
        }
        // bytes < TAG_BUSY (empty or dead): high bit of (byte - 2) with the byte's high bit clear
        const uint64_t fr = ((tags | highs) - 2 * ones) ^ highs;
        const uint64_t freeb = fr & ~tags & highs & valid;
        if (!have_free && freeb) { have_free = true; fb = b; ftags = tags; }
        if (empty || (known_absent && have_free)) break;
        b = (b + 1) & t.mask;
    }
    if (!have_free) return -1;                                     // S::MAXP full buckets
    b = fb;
    for (int p = 0; p < S::MAXP; ++p) {                          // 2) claim (one CAS per try)
        CV_G uint32_t *bw = G(t.buckets) + b * S::BW;
        uint64_t cur = ftags;
        if (p > 0) {
            const uint2 tg = make_uint2(__hip_atomic_load(bw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                        __hip_atomic_load(bw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            cur = (uint64_t)tg.x | ((uint64_t)tg.y << 32);
        }
        int got = -1;
        uint32_t old = TAG_DEAD;
        if (claim_in_word(bw, (uint32_t)cur, 0, S::SPB < 4 ? S::SPB : 4, tag, got, old) ||
            (S::SPB > 4 && claim_in_word(bw + 1, (uint32_t)(cur >> 32), 4, S::SPB - 4, tag, got, old))) {
            if (was) *was = old;                                  // (the claimed slot's tag: empty or dead)
#pragma unroll
            for (int j = 0; j < S::KW; ++j) bw[S::KEY0 + got * S::KS + j] = key[j];
            *created = true;
            return (int64_t)(b * S::SPB + got);
        }
        b = (b + 1) & t.mask;
    }
    return -1;
}

// Conntrack delete (map_delete_elem, conntrack.h:641-647): key and value slot -> zero
// words, then tag -> dead.  The clearing writes are agent-scope atomics and complete
// (the workgroup-scope release waits for them, without an L2 write-back) before the
// tag CAS is issued.  A later claim of the dead slot in the same launch may come from
// another XCD, whose L2 is not coherent with this one: the atomics leave no dirty
// copy of the slot's key or value line in this XCD's L2 that the kernel-end write-back
// could lay over the new owner's entry.
template <class S>
__device__ __forceinline__ void dev_kill(const HashTable &t, int64_t slot)
{
    const uint64_t b = (uint64_t)slot / S::SPB;
    const int s = (int)((uint64_t)slot % S::SPB);
    CV_G uint32_t *tw = G(t.buckets) + b * S::BW + (s >> 2);
    const int sh = 8 * (s & 3);
#pragma unroll
    for (int j = 0; j < S::KS; ++j)                               // the key, and a CT slot's hot words
        __hip_atomic_exchange(G(t.buckets) + b * S::BW + S::KEY0 + s * S::KS + j, 0u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    if (t.vals) {
        CV_G unsigned long long *v = reinterpret_cast<CV_G unsigned long long *>(G(t.vals) + (size_t)slot * t.vstride);
        for (uint32_t j = 0; j < t.vstride / 8; ++j)
            __hip_atomic_store(v + j, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t c = __hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        const uint32_t n = (c & ~(0xFFu << sh)) | (TAG_DEAD << sh);
        if (__hip_atomic_compare_exchange_strong(tw, &c, n, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            break;
    }
}

// ---------------------------------------------------------------- host build
template <class S>
inline uint32_t *host_bucket(HashTable &t, uint64_t b) { return t.buckets + b * S::BW; }

template <class S>
inline void host_set_ival(uint32_t *w, int s, const uint32_t *ival)
{
    for (int j = 0; j < S::IVW; ++j) w[S::IVAL0 + s * S::IVW + j] = ival ? ival[j] : 0;
    if (S::IVH) {
        const int h = S::HVAL0 + s, sh = 16 * (h & 1);
        w[h >> 1] = (w[h >> 1] & ~(0xFFFFu << sh)) | ((ival ? ival[0] & 0xFFFFu : 0u) << sh);
    }
}

// Insert or overwrite on a host copy.  Returns slot, or -1 when the chain is longer
// than S::MAXP (caller grows the table).
template <class S>
inline int64_t host_upsert(HashTable &t, const uint32_t *key, const uint32_t *ival)
{
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    uint64_t b = h & t.mask;
    int64_t free_slot = -1;
    for (int p = 0; p < S::MAXP; ++p) {
        uint32_t *w = host_bucket<S>(t, b);
        bool stop;
        int s = match_bucket<S>(w, key, tag, &stop);
        if (s >= 0) {
            host_set_ival<S>(w, s, ival);
            return (int64_t)(b * S::SPB + s);
        }
        if (free_slot < 0) {
            uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
            for (int q = 0; q < S::SPB; ++q)
                if (((tags >> (8 * q)) & 0xFF) < TAG_BUSY) { free_slot = (int64_t)(b * S::SPB + q); break; }
        }
        if (stop) break;
        b = (b + 1) & t.mask;
    }
    if (free_slot < 0) return -1;
    uint64_t fb = (uint64_t)free_slot / S::SPB;
    int q = (int)((uint64_t)free_slot % S::SPB);
    uint32_t *w = host_bucket<S>(t, fb);
    for (int j = 0; j < S::KW; ++j) w[S::KEY0 + q * S::KS + j] = key[j];
    host_set_ival<S>(w, q, ival);
    uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    tags = (tags & ~(0xFFULL << (8 * q))) | ((uint64_t)tag << (8 * q));
    w[0] = (uint32_t)tags; w[1] = (uint32_t)(tags >> 32);
    return free_slot;
}

template <class S>
inline int64_t host_find(const HashTable &t, const uint32_t *key)
{
    uint32_t tag;
    const uint64_t h = home_hash<S>(key, tag);
    uint64_t b = h & t.mask;
    for (int p = 0; p < S::MAXP; ++p) {
        const uint32_t *w = t.buckets + b * S::BW;
        bool stop;
        int s = match_bucket<S>(w, key, tag, &stop);
        if (s >= 0) return (int64_t)(b * S::SPB + s);
        if (stop) return -1;
        b = (b + 1) & t.mask;
    }
    return -1;
}

inline uint64_t buckets_for(uint64_t n, int spb, double load = 0.6)
{
    uint64_t need = (uint64_t)((double)(n ? n : 1) / (spb * load)) + 1, nb = 16;
    while (nb < need) nb <<= 1;
    return nb;
}

}  // namespace cv
