// cv_lpm.hpp — longest-prefix-match tables (the LPM_TRIE maps of the reference:
// cilium_ipcache, v4_dyn / v6_dyn prefilter maps).
//
// IPv4: a 16-8-8 multibit trie with leaf pushing, compiled on the host from the
// map's prefixes in increasing prefix-length order (so a longer prefix overrides
// the slots of every shorter one it covers, exactly the kernel LPM_TRIE answer,
// kernel/bpf/lpm_trie.c trie_lookup_elem).  Every slot holds the final answer:
//   bit31 = 1  -> child chunk index (bits 0..30), 256 slots per chunk
//   otherwise  -> the value of the longest matching prefix (0 = no match)
// L1 has 65536 slots (256 KiB, L2-resident); a lookup is 1-3 dependent 4-B reads.
//
// IPv6 (and any prefix outside the trie's reach): one hash table keyed by
// (masked address, prefix length) probed from the longest stored length down:
// the same answer, one line read per distinct length tried.
#pragma once
#include <algorithm>
#include <vector>

#include "cv_hash.hpp"

namespace cv {

struct Lpm4 {                  // POD device view
    const uint32_t *l1;        // 65536 slots
    const uint32_t *chunks;    // nchunks * 256 slots
    HashTable full;            // optional /32 front (Host32Spec): a /32 is always the longest
                               // match, so a hit ends the lookup in one L2-resident line
};

using Host32Spec = HashSpec<1, 1, 7, 16>;   // raw ip4 -> value

__device__ __forceinline__ uint32_t lpm4_lookup(const Lpm4 &t, uint32_t addr /* host order */)
{
    if (t.full.buckets) {
        const uint32_t k = bswap32(addr);
        uint32_t v;
        if (dev_find<Host32Spec>(t.full, &k, &v) >= 0) return v;
    }
    uint32_t e = t.l1[addr >> 16];
    if (e & 0x80000000u) {
        e = t.chunks[((e & 0x7FFFFFFFu) << 8) | ((addr >> 8) & 0xFFu)];
        if (e & 0x80000000u) e = t.chunks[((e & 0x7FFFFFFFu) << 8) | (addr & 0xFFu)];
    }
    return e;
}

// lpm4_lookup with the /32 front read by a quad probe: every lane of the wave calls
// it; returns 0 when `want` is false
__device__ __forceinline__ uint32_t lpm4_lookup_q(const Lpm4 &t, uint32_t addr /* host order */, bool want, uint4 *st)
{
    const uint32_t k = bswap32(addr);
    uint32_t v = 0;
    if (t.full.buckets && quad_find<Host32Spec>(t.full, &k, want, st, &v) >= 0) return v;   // (uniform test)
    if (!want) return 0;
    uint32_t e = t.l1[addr >> 16];                                // (prefetching it beside the front: +2 %)
    if (e & 0x80000000u) {
        e = t.chunks[((e & 0x7FFFFFFFu) << 8) | ((addr >> 8) & 0xFFu)];
        if (e & 0x80000000u) e = t.chunks[((e & 0x7FFFFFFFu) << 8) | (addr & 0xFFu)];
    }
    return e;
}

// The same answer with the /32-front probe and the trie's first level read issued
// together (one round trip when the front hits or the level-1 slot is final).
struct Lpm4Pending {
    Probe<Host32Spec> front;
    uint32_t l1;
    uint32_t addr;
};

__device__ __forceinline__ Lpm4Pending lpm4_begin(const Lpm4 &t, uint32_t addr /* host order */)
{
    Lpm4Pending q;
    q.addr = addr;
    const uint32_t k = bswap32(addr);
    q.front = probe_begin<Host32Spec>(t.full, &k);
    q.l1 = t.l1[addr >> 16];
    return q;
}

__device__ __forceinline__ uint32_t lpm4_end(const Lpm4Pending &q, const Lpm4 &t)
{
    if (t.full.buckets) {
        const uint32_t k = bswap32(q.addr);
        uint32_t v;
        if (probe_end<Host32Spec>(q.front, t.full, &k, &v) >= 0) return v;
    }
    uint32_t e = q.l1;
    if (e & 0x80000000u) {
        e = t.chunks[((e & 0x7FFFFFFFu) << 8) | ((q.addr >> 8) & 0xFFu)];
        if (e & 0x80000000u) e = t.chunks[((e & 0x7FFFFFFFu) << 8) | (q.addr & 0xFFu)];
    }
    return e;
}

// Host builder.  Prefixes must be fed in non-decreasing priority (prefix length).
struct Lpm4Builder {
    std::vector<uint32_t> l1 = std::vector<uint32_t>(65536, 0);
    std::vector<uint32_t> chunks;
    std::vector<uint32_t> free_chunks;         // chunks of rebuilt subtrees, reused first
    std::vector<uint32_t> touched;             // chunks written since the last take_touched()

    uint32_t new_chunk(uint32_t fill)
    {
        uint32_t idx;
        if (!free_chunks.empty()) {
            idx = free_chunks.back();
            free_chunks.pop_back();
            std::fill(chunks.begin() + (size_t)idx * 256, chunks.begin() + (size_t)idx * 256 + 256, fill);
        } else {
            idx = (uint32_t)(chunks.size() / 256);
            chunks.insert(chunks.end(), 256, fill);
        }
        touched.push_back(idx);
        return idx;
    }

    // the chunks under a level-1 slot to the free list (the slot is about to be rebuilt)
    void release(uint32_t e)
    {
        if (!(e & 0x80000000u)) return;
        const uint32_t c2 = e & 0x7FFFFFFFu;
        for (uint32_t i = 0; i < 256; ++i) {
            const uint32_t e2 = chunks[((size_t)c2 << 8) + i];
            if (e2 & 0x80000000u) free_chunks.push_back(e2 & 0x7FFFFFFFu);
        }
        free_chunks.push_back(c2);
    }

    // value must be < 2^31 (0 = no match)
    void insert(uint32_t addr, int plen, uint32_t value)
    {
        if (plen <= 16) {
            uint32_t span = 1u << (16 - plen);
            uint32_t base = plen == 0 ? 0 : (addr >> 16) & ~(span - 1);
            for (uint32_t i = 0; i < span; ++i) fill_slot(&l1[base + i], value, 1);
            return;
        }
        uint32_t *s1 = &l1[addr >> 16];
        if (!(*s1 & 0x80000000u)) *s1 = 0x80000000u | new_chunk(*s1);
        uint32_t c2 = *s1 & 0x7FFFFFFFu;
        if (plen <= 24) {
            uint32_t span = 1u << (24 - plen);
            uint32_t base = ((addr >> 8) & 0xFFu) & ~(span - 1);
            for (uint32_t i = 0; i < span; ++i) fill_slot(&chunks[(c2 << 8) + base + i], value, 2);
            return;
        }
        uint32_t *s2 = &chunks[(c2 << 8) | ((addr >> 8) & 0xFFu)];
        if (!(*s2 & 0x80000000u)) {
            uint32_t nc = new_chunk(*s2);
            s2 = &chunks[(c2 << 8) | ((addr >> 8) & 0xFFu)];   // vector may have moved
            *s2 = 0x80000000u | nc;
        }
        uint32_t c3 = *s2 & 0x7FFFFFFFu;
        uint32_t span = 1u << (32 - plen);
        uint32_t base = (addr & 0xFFu) & ~(span - 1);
        for (uint32_t i = 0; i < span; ++i) chunks[(c3 << 8) + base + i] = value;
    }

  private:
    // A prefix inserted later (longer or equal priority) overrides a slot; when the
    // slot already points to a child (only possible for equal-priority re-insert of
    // an overlapping range), push the value into the child's slots.
    void fill_slot(uint32_t *s, uint32_t value, int level)
    {
        if (!(*s & 0x80000000u)) { *s = value; return; }
        uint32_t c = *s & 0x7FFFFFFFu;
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t *t = &chunks[(c << 8) + i];
            if (level == 1) fill_slot(t, value, 2);
            else if (!(*t & 0x80000000u)) *t = value;
            else fill_slot(t, value, 3);
        }
    }
};

// v6 / generic LPM as (masked address, plen) hash + descending list of lengths
struct Lpm6 {
    HashTable h;               // Lpm6Spec: key = 4 address words (masked) + plen
    const uint8_t *lens;       // distinct prefix lengths, descending
    uint32_t nlens;
};

__device__ __forceinline__ void mask128(const uint32_t *a, int plen, uint32_t *o)
{
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        int bits = plen - 32 * w;
        uint32_t m = bits <= 0 ? 0u : bits >= 32 ? 0xFFFFFFFFu : bswap32(0xFFFFFFFFu << (32 - bits));
        o[w] = a[w] & m;
    }
}

// `a` = 16 address bytes as 4 raw (network-order) words; returns value or 0
__device__ __forceinline__ uint32_t lpm6_lookup(const Lpm6 &t, const uint32_t *a)
{
    for (uint32_t i = 0; i < t.nlens; ++i) {
        const int plen = t.lens[i];
        uint32_t k[5];
        mask128(a, plen, k);
        k[4] = (uint32_t)plen;
        uint32_t v;
        if (dev_find<Lpm6Spec>(t.h, k, &v) >= 0) return v;
    }
    return 0;
}

}  // namespace cv
