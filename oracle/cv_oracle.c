/*
 * cv_oracle.c — CPU restatement of Cilium's L3/L4 verdict path (TEST INFRASTRUCTURE).
 * See cv_oracle.h.  Reference = Taeung/cilium v1.1.90 under /root/reference.
 * Restated, not copied: every block cites the reference lines it follows.
 */
#include "cv_oracle.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

/* ===================================================================== */
/* Kernel map semantics                                                   */
/* HASH: kernel/bpf/hashtab.c htab_map_update_elem: flags > BPF_EXIST ->  */
/*   -EINVAL; NOEXIST on existing -> -EEXIST; EXIST on missing ->         */
/*   -ENOENT; new element when count == max_entries -> -E2BIG.            */
/* LPM_TRIE: kernel/bpf/lpm_trie.c: a key is (prefixlen, first prefixlen  */
/*   bits of data); prefixlen > max -> -EINVAL; full -> -ENOSPC; lookup   */
/*   returns the longest stored prefix whose prefixlen <= the lookup key's */
/*   prefixlen and whose bits match; delete is exact.                     */
/* ===================================================================== */

typedef struct {
    uint32_t ks, vs, cap, count;
    uint8_t *keys, *vals, *used;
} or_hash;

static uint64_t hbytes(const uint8_t *k, uint32_t n)
{
    uint64_t h = 1469598103934665603ULL;
    for (uint32_t i = 0; i < n; i++) { h ^= k[i]; h *= 1099511628211ULL; }
    h ^= h >> 33; h *= 0xff51afd7ed558ccdULL; h ^= h >> 33;
    return h;
}

static or_hash *hnew(uint32_t ks, uint32_t vs, uint32_t cap)
{
    or_hash *h = calloc(1, sizeof(*h));
    uint32_t c = 16;
    while (c < cap) c <<= 1;
    h->ks = ks; h->vs = vs; h->cap = c;
    h->keys = calloc((size_t)c, ks);
    h->vals = calloc((size_t)c, vs ? vs : 1);
    h->used = calloc(c, 1);
    return h;
}

static void hfree(or_hash *h)
{
    if (!h) return;
    free(h->keys); free(h->vals); free(h->used); free(h);
}

static int64_t hfind(const or_hash *h, const uint8_t *k)
{
    uint32_t m = h->cap - 1, i = (uint32_t)hbytes(k, h->ks) & m;
    while (h->used[i]) {
        if (!memcmp(h->keys + (size_t)i * h->ks, k, h->ks)) return i;
        i = (i + 1) & m;
    }
    return -1;
}

static void hgrow(or_hash *h)
{
    or_hash *n = hnew(h->ks, h->vs, h->cap * 2);
    for (uint32_t i = 0; i < h->cap; i++) {
        if (!h->used[i]) continue;
        uint32_t m = n->cap - 1, j = (uint32_t)hbytes(h->keys + (size_t)i * h->ks, h->ks) & m;
        while (n->used[j]) j = (j + 1) & m;
        n->used[j] = 1;
        memcpy(n->keys + (size_t)j * h->ks, h->keys + (size_t)i * h->ks, h->ks);
        memcpy(n->vals + (size_t)j * h->vs, h->vals + (size_t)i * h->vs, h->vs);
    }
    n->count = h->count;
    free(h->keys); free(h->vals); free(h->used);
    *h = *n; free(n);
}

/* returns slot of key, inserting a zero value if missing */
static int64_t hput(or_hash *h, const uint8_t *k)
{
    int64_t s = hfind(h, k);
    if (s >= 0) return s;
    if ((h->count + 1) * 2 > h->cap) hgrow(h);
    uint32_t m = h->cap - 1, i = (uint32_t)hbytes(k, h->ks) & m;
    while (h->used[i]) i = (i + 1) & m;
    h->used[i] = 1; h->count++;
    memcpy(h->keys + (size_t)i * h->ks, k, h->ks);
    memset(h->vals + (size_t)i * h->vs, 0, h->vs);
    return i;
}

static void hdel_slot(or_hash *h, uint32_t i)
{   /* backward-shift deletion for linear probing */
    uint32_t m = h->cap - 1, j = i;
    h->used[i] = 0; h->count--;
    for (;;) {
        j = (j + 1) & m;
        if (!h->used[j]) break;
        uint32_t k = (uint32_t)hbytes(h->keys + (size_t)j * h->ks, h->ks) & m;
        int move = (j > i) ? (k <= i || k > j) : (k <= i && k > j);
        if (move) {
            memcpy(h->keys + (size_t)i * h->ks, h->keys + (size_t)j * h->ks, h->ks);
            memcpy(h->vals + (size_t)i * h->vs, h->vals + (size_t)j * h->vs, h->vs);
            h->used[i] = 1; h->used[j] = 0;
            i = j;
        }
    }
}

struct or_map {
    int type;
    uint32_t ks, vs, max;
    or_hash *h;              /* HASH / LRU_HASH */
    uint32_t dbits;          /* LPM: data bits */
    or_hash **lpm;           /* LPM: per prefixlen, key = masked data, val = orig data + value */
    uint32_t lpm_count;
};

or_map *or_map_create(int type, uint32_t key_size, uint32_t val_size, uint32_t max_entries)
{
    if (!key_size || !max_entries) return NULL;
    or_map *m = calloc(1, sizeof(*m));
    m->type = type; m->ks = key_size; m->vs = val_size; m->max = max_entries;
    if (type == OR_MAP_LPM_TRIE) {
        if (key_size <= 4) { free(m); return NULL; }
        m->dbits = (key_size - 4) * 8;
        m->lpm = calloc(m->dbits + 1, sizeof(or_hash *));
    } else {
        m->h = hnew(key_size, val_size, 64);
    }
    return m;
}

void or_map_free(or_map *m)
{
    if (!m) return;
    hfree(m->h);
    if (m->lpm) {
        for (uint32_t i = 0; i <= m->dbits; i++) hfree(m->lpm[i]);
        free(m->lpm);
    }
    free(m);
}

static void mask_bits(uint8_t *d, uint32_t nbytes, uint32_t plen)
{
    for (uint32_t b = 0; b < nbytes; b++) {
        uint32_t lo = b * 8;
        if (plen >= lo + 8) continue;
        d[b] = plen <= lo ? 0 : (uint8_t)(d[b] & (0xFF00u >> (plen - lo)));
    }
}

int or_map_update(or_map *m, const void *key, const void *val, uint64_t flags)
{
    if (flags > OR_BPF_EXIST) return -EINVAL;
    if (m->type == OR_MAP_LPM_TRIE) {
        uint32_t plen; memcpy(&plen, key, 4);
        uint32_t nb = m->ks - 4;
        if (plen > m->dbits) return -EINVAL;
        uint8_t mk[64]; memcpy(mk, (const uint8_t *)key + 4, nb); mask_bits(mk, nb, plen);
        if (!m->lpm[plen]) m->lpm[plen] = hnew(nb, nb + m->vs, 16);
        int64_t s = hfind(m->lpm[plen], mk);
        if (s >= 0) {
            if (flags == OR_BPF_NOEXIST) return -EEXIST;
        } else {
            if (flags == OR_BPF_EXIST) return -ENOENT;
            if (m->lpm_count >= m->max) return -ENOSPC;
            s = hput(m->lpm[plen], mk);
            m->lpm_count++;
        }
        uint8_t *v = m->lpm[plen]->vals + (size_t)s * (nb + m->vs);
        memcpy(v, (const uint8_t *)key + 4, nb);
        memcpy(v + nb, val, m->vs);
        return 0;
    }
    int64_t s = hfind(m->h, key);
    if (s >= 0) {
        if (flags == OR_BPF_NOEXIST) return -EEXIST;
    } else {
        if (flags == OR_BPF_EXIST) return -ENOENT;
        if (m->h->count >= m->max) return -E2BIG;
        s = hput(m->h, key);
    }
    memcpy(m->h->vals + (size_t)s * m->vs, val, m->vs);
    return 0;
}

int or_map_update_batch(or_map *m, const void *keys, const void *vals, uint32_t n, uint64_t flags)
{
    for (uint32_t i = 0; i < n; i++) {
        int r = or_map_update(m, (const uint8_t *)keys + (size_t)i * m->ks, (const uint8_t *)vals + (size_t)i * m->vs,
                              flags);
        if (r) return r;
    }
    return 0;
}

void *or_map_lookup_ptr(or_map *m, const void *key)
{
    if (m->type == OR_MAP_LPM_TRIE) {
        uint32_t plen; memcpy(&plen, key, 4);
        uint32_t nb = m->ks - 4;
        if (plen > m->dbits) plen = m->dbits;
        for (int l = (int)plen; l >= 0; l--) {
            if (!m->lpm[l] || !m->lpm[l]->count) continue;
            uint8_t mk[64]; memcpy(mk, (const uint8_t *)key + 4, nb); mask_bits(mk, nb, (uint32_t)l);
            int64_t s = hfind(m->lpm[l], mk);
            if (s >= 0) return m->lpm[l]->vals + (size_t)s * (nb + m->vs) + nb;
        }
        return NULL;
    }
    int64_t s = hfind(m->h, key);
    return s >= 0 ? m->h->vals + (size_t)s * m->vs : NULL;
}

int or_map_lookup(or_map *m, const void *key, void *val_out)
{
    void *p = or_map_lookup_ptr(m, key);
    if (!p) return -ENOENT;
    if (val_out) memcpy(val_out, p, m->vs);
    return 0;
}

int or_map_delete(or_map *m, const void *key)
{
    if (m->type == OR_MAP_LPM_TRIE) {
        uint32_t plen; memcpy(&plen, key, 4);
        uint32_t nb = m->ks - 4;
        if (plen > m->dbits || !m->lpm[plen]) return -ENOENT;
        uint8_t mk[64]; memcpy(mk, (const uint8_t *)key + 4, nb); mask_bits(mk, nb, plen);
        int64_t s = hfind(m->lpm[plen], mk);
        if (s < 0) return -ENOENT;
        hdel_slot(m->lpm[plen], (uint32_t)s);
        m->lpm_count--;
        return 0;
    }
    int64_t s = hfind(m->h, key);
    if (s < 0) return -ENOENT;
    hdel_slot(m->h, (uint32_t)s);
    return 0;
}

uint32_t or_map_count(const or_map *m)
{
    return m->type == OR_MAP_LPM_TRIE ? m->lpm_count : m->h->count;
}

static uint32_t g_sort_ks;
static int cmp_rows(const void *a, const void *b) { return memcmp(a, b, g_sort_ks); }

/* Order-independent digest of a hash map's entries (test infrastructure: compares a
 * 33M-entry conntrack table with the device's without sorting either dump).  Per
 * entry: the key then the value, each zero-padded to 8-byte words, chained through
 * splitmix64's finalizer from a fixed seed; out = {count, sum of the chains mod 2^64,
 * xor of the chains}.  tests/harness.table_digest is the same function over dumps. */
static uint64_t dg_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static uint64_t dg_row(const uint8_t *k, uint32_t ks, const uint8_t *v, uint32_t vs)
{
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (int part = 0; part < 2; part++) {
        const uint8_t *p = part ? v : k;
        uint32_t n = part ? vs : ks;
        for (uint32_t o = 0; o < n; o += 8) {
            uint64_t w = 0;
            memcpy(&w, p + o, n - o < 8 ? n - o : 8);
            h = dg_mix(h ^ w);
        }
    }
    return h;
}

void or_map_digest(const or_map *m, uint64_t out[3])
{
    uint64_t cnt = 0, sum = 0, x = 0;
    if (m->type != OR_MAP_LPM_TRIE) {
        for (uint32_t i = 0; i < m->h->cap; i++) {
            if (!m->h->used[i]) continue;
            const uint64_t h = dg_row(m->h->keys + (size_t)i * m->ks, m->ks, m->h->vals + (size_t)i * m->vs, m->vs);
            cnt++; sum += h; x ^= h;
        }
    }
    out[0] = cnt; out[1] = sum; out[2] = x;
}

uint32_t or_map_dump(const or_map *m, void *keys, void *vals, uint32_t max)
{
    uint32_t n = or_map_count(m), row = m->ks + m->vs, k = 0;
    uint8_t *tmp = malloc((size_t)(n ? n : 1) * row);
    if (m->type == OR_MAP_LPM_TRIE) {
        uint32_t nb = m->ks - 4;
        for (uint32_t l = 0; l <= m->dbits; l++) {
            or_hash *h = m->lpm[l];
            if (!h) continue;
            for (uint32_t i = 0; i < h->cap; i++) {
                if (!h->used[i]) continue;
                uint8_t *r = tmp + (size_t)k++ * row;
                memcpy(r, &l, 4);
                memcpy(r + 4, h->vals + (size_t)i * (nb + m->vs), nb + m->vs);
            }
        }
    } else {
        for (uint32_t i = 0; i < m->h->cap; i++) {
            if (!m->h->used[i]) continue;
            uint8_t *r = tmp + (size_t)k++ * row;
            memcpy(r, m->h->keys + (size_t)i * m->ks, m->ks);
            memcpy(r + m->ks, m->h->vals + (size_t)i * m->vs, m->vs);
        }
    }
    g_sort_ks = m->ks;
    qsort(tmp, k, row, cmp_rows);
    if (k > max) k = max;
    for (uint32_t i = 0; i < k; i++) {
        if (keys) memcpy((uint8_t *)keys + (size_t)i * m->ks, tmp + (size_t)i * row, m->ks);
        if (vals) memcpy((uint8_t *)vals + (size_t)i * m->vs, tmp + (size_t)i * row + m->ks, m->vs);
    }
    free(tmp);
    return k;
}

/* ===================================================================== */
/* Byte order + helpers                                                   */
/* ===================================================================== */

static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* GET_PREFIX (bpf/lib/ipv6.h:136-138), evaluated in int arithmetic as the macro does */
uint32_t or_get_prefix(int prefix)
{
    uint32_t host = prefix <= 0 ? 0u : prefix < 32 ? (uint32_t)(((1u << prefix) - 1u) << (32 - prefix))
                                                   : 0xFFFFFFFFu;
    return bswap32(host);
}

/* ipv6_addr_clear_suffix (bpf/lib/ipv6.h:140-150) */
void or_ipv6_addr_clear_suffix(uint8_t addr[16], int prefix)
{
    for (int w = 0; w < 4; w++) {
        uint32_t p; memcpy(&p, addr + 4 * w, 4);
        p &= or_get_prefix(prefix);
        memcpy(addr + 4 * w, &p, 4);
        prefix -= 32;
    }
}

/* skb_load_bytes / direct access bound: bytes [off, off+n) must lie inside skb->len.
 * `avail` = bytes present in the record (min(len, stride)).  Returns 0, 1 (beyond
 * len: the reference's helper fails) or OR_E_TRUNC (inside len but not in the record). */
static inline int ld(const uint8_t *f, uint32_t avail, uint32_t len, int off, uint32_t n, void *to)
{
    if (off < 0 || (uint64_t)off + n > len) return 1;
    if ((uint64_t)off + n > avail) return OR_E_TRUNC;
    memcpy(to, f + off, n);
    return 0;
}

#define ETH_HLEN 14
#define HOST_ID 1     /* bpf/node_config.h */
#define WORLD_ID 2
#define CLUSTER_ID 3
#define HEALTH_ID 4
#define HOST_IFINDEX 1

/* ===================================================================== */
/* Datapath container                                                     */
/* ===================================================================== */

or_dp *or_dp_create(uint32_t flags)
{
    or_dp *dp = calloc(1, sizeof(*dp));
    dp->flags = flags;
    return dp;
}

void or_dp_free(or_dp *dp) { free(dp); }

int or_dp_endpoint_config(or_dp *dp, uint32_t ep, uint32_t ipv4, const uint8_t *ipv6, const uint8_t *mac,
                          const uint8_t *node_mac, or_map *ct6)
{
    if (ep >= dp->n_ep) return -EINVAL;
    or_endpoint_prog *e = &dp->ep[ep];
    e->ipv4 = ipv4;
    if (ipv6) memcpy(e->ipv6, ipv6, 16);
    if (mac) memcpy(e->mac, mac, 6);
    if (node_mac) memcpy(e->node_mac, node_mac, 6);
    e->ct6 = ct6;
    return 0;
}

void or_dp_node_config(or_dp *dp, uint32_t mask, uint32_t range, uint32_t loopback, const uint8_t *router_ip6,
                       const uint8_t *host_mac, const uint8_t *net_mac)
{
    dp->v4_cluster_mask = mask; dp->v4_cluster_range = range; dp->v4_loopback = loopback;
    if (router_ip6) memcpy(dp->router_ip6, router_ip6, 16);
    if (host_mac) memcpy(dp->host_mac, host_mac, 6);
    if (net_mac) memcpy(dp->net_mac, net_mac, 6);
}

int or_dp_add_endpoint(or_dp *dp, uint16_t lxc_id, uint32_t seclabel, or_map *policy, or_map *ct4)
{
    if (dp->n_ep >= OR_MAX_EP) return -E2BIG;
    or_endpoint_prog *e = &dp->ep[dp->n_ep];
    e->lxc_id = lxc_id; e->seclabel = seclabel; e->policy = policy; e->ct4 = ct4;
    dp->ep_of_lxc[lxc_id] = (uint16_t)(dp->n_ep + 1);
    return (int)dp->n_ep++;
}

void or_dp_metrics(const or_dp *dp, uint64_t *out) { memcpy(out, dp->metrics, sizeof(dp->metrics)); }

void or_dp_notify_attach(or_dp *dp, or_drop_notify *buf, uint32_t cap)
{
    dp->notify = buf;
    dp->notify_cap = buf ? cap : 0;
    dp->notify_n = 0;
}

uint32_t or_dp_notify_count(const or_dp *dp) { return dp->notify_n; }

void or_dp_trace_attach(or_dp *dp, or_trace_notify *buf, uint32_t cap, uint32_t aggregation, uint32_t ingress_ifindex)
{
    dp->trace = buf;
    dp->trace_cap = buf ? cap : 0;
    dp->trace_n = 0;
    dp->trace_agg = aggregation;
    dp->ingress_ifindex = ingress_ifindex;
}

uint32_t or_dp_trace_count(const or_dp *dp) { return dp->trace_n; }

/* observation points and aggregation levels (bpf/lib/trace.h:38-62) */
enum { TRACE_TO_LXC, TRACE_TO_PROXY, TRACE_TO_HOST, TRACE_TO_STACK, TRACE_TO_OVERLAY,
       TRACE_FROM_LXC, TRACE_FROM_PROXY, TRACE_FROM_HOST, TRACE_FROM_STACK, TRACE_FROM_OVERLAY };
#define TRACE_AGGREGATE_RX 1
#define TRACE_AGGREGATE_ACTIVE_CT 3

/* send_trace_notify (bpf/lib/trace.h:96-150), TRACE_NOTIFY on (lxc_config.h:36): the
 * cilium_events record of a forwarding step; the update_metrics half is the caller's.
 * FROM_* points are hidden at MONITOR_AGGREGATION >= RX, and everything the CT marked
 * as not worth a report (monitor false) at >= ACTIVE_CT. */
static void notify_trace(or_dp *dp, uint8_t obs, uint32_t len, uint16_t source, uint32_t src, uint32_t dst,
                         uint16_t dst_id, uint32_t ifindex, uint8_t reason, int monitor)
{
    if (!dp->trace) return;
    if (dp->trace_agg >= TRACE_AGGREGATE_RX && obs >= TRACE_FROM_LXC) return;
    if (dp->trace_agg >= TRACE_AGGREGATE_ACTIVE_CT && !monitor) return;
    const uint32_t at = dp->trace_n++;
    if (at >= dp->trace_cap) return;
    or_trace_notify *m = &dp->trace[at];
    m->type = 4;                                   /* CILIUM_NOTIFY_TRACE (common.h:209-215) */
    m->subtype = obs;
    m->source = source;
    m->hash = dp->cur_hash;
    m->len_orig = len;
    m->len_cap = len < 128 ? len : 128;
    m->src_label = src;
    m->dst_label = dst;
    m->dst_id = dst_id;
    m->reason = reason;
    m->pad = 0;
    m->ifindex = ifindex;
    m->packet = dp->cur_pkt;
    m->reserved = 0;
}

/* send_drop_notify (bpf/lib/drop.h:94-108) -> __send_drop_notify (:50-79): the
 * cilium_events record of a drop; cb[1] = src << 16 | (dst & 0xFFFF) is split back into
 * 16-bit labels; subtype = -reason; source = EVENT_SOURCE of the program (LXC_ID in
 * bpf_lxc, 0 in bpf_netdev); the update_metrics half is the caller's. */
static void notify_drop(or_dp *dp, int reason, uint32_t len, uint16_t source, uint32_t src, uint32_t dst,
                        uint32_t dst_id, uint32_t ifindex)
{
    if (!dp->notify) return;
    const uint32_t at = dp->notify_n++;
    if (at >= dp->notify_cap) return;
    or_drop_notify *m = &dp->notify[at];
    const uint32_t srcdst = (src << 16) | (dst & 0xFFFFu);
    m->type = 1;                                   /* CILIUM_NOTIFY_DROP */
    m->subtype = (uint8_t)(reason < 0 ? -reason : reason);
    m->source = source;
    m->hash = dp->cur_hash;
    m->len_orig = len;
    m->len_cap = len < 128 ? len : 128;            /* TRACE_PAYLOAD_LEN */
    m->src_label = srcdst >> 16;
    m->dst_label = srcdst & 0xFFFFu;
    m->dst_id = dst_id;
    m->ifindex = ifindex;
    m->packet = dp->cur_pkt;
    m->reserved = 0;
}

/* update_metrics (bpf/lib/metrics.h:43-58) summed over CPUs; dir 1 ingress, 2 egress */
static void update_metrics(or_dp *dp, uint32_t bytes, uint8_t dir, uint8_t reason)
{
    __atomic_fetch_add(&dp->metrics[reason][dir & 3][0], 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&dp->metrics[reason][dir & 3][1], (uint64_t)bytes, __ATOMIC_RELAXED);
}

static or_endpoint_prog *find_ep(or_dp *dp, uint16_t lxc_id)
{
    uint16_t e = dp->ep_of_lxc[lxc_id];
    return e ? &dp->ep[e - 1] : NULL;
}

/* lookup_ip4_endpoint / lookup_ip6_endpoint (bpf/lib/eps.h:26-46) */
static or_endpoint_info *lookup_ip4_endpoint(or_dp *dp, uint32_t daddr, uint8_t *nl)
{
    if (!dp->lxc) return NULL;
    or_endpoint_key k; memset(&k, 0, sizeof(k));
    memcpy(k.ip, &daddr, 4); k.family = 1;
    (*nl)++;
    return or_map_lookup_ptr(dp->lxc, &k);
}

static or_endpoint_info *lookup_ip6_endpoint(or_dp *dp, const uint8_t *daddr, uint8_t *nl)
{
    if (!dp->lxc) return NULL;
    or_endpoint_key k; memset(&k, 0, sizeof(k));
    memcpy(k.ip, daddr, 16); k.family = 2;
    (*nl)++;
    return or_map_lookup_ptr(dp->lxc, &k);
}

/* ipcache_lookup4 (bpf/lib/eps.h:68-86) with prefix = V4_CACHE_KEY_LEN (32):
 * key.lpm prefixlen = IPCACHE_PREFIX_LEN(32) = 32 static bits + 32. */
static or_remote_endpoint_info *ipcache_lookup4(or_dp *dp, uint32_t addr, int prefix, uint8_t *nl)
{
    if (!dp->ipcache) return NULL;
    or_ipcache_key k; memset(&k, 0, sizeof(k));
    k.prefixlen = 32 + (uint32_t)prefix; k.family = 1;
    addr &= or_get_prefix(prefix);
    memcpy(k.ip, &addr, 4);
    (*nl)++;
    return or_map_lookup_ptr(dp->ipcache, &k);
}

/* ipcache_lookup6 (bpf/lib/eps.h:54-66) */
static or_remote_endpoint_info *ipcache_lookup6(or_dp *dp, const uint8_t *addr, int prefix, uint8_t *nl)
{
    if (!dp->ipcache) return NULL;
    or_ipcache_key k; memset(&k, 0, sizeof(k));
    k.prefixlen = 32 + (uint32_t)prefix; k.family = 2;
    memcpy(k.ip, addr, 16);
    or_ipv6_addr_clear_suffix(k.ip, prefix);
    (*nl)++;
    return or_map_lookup_ptr(dp->ipcache, &k);
}

/* ===================================================================== */
/* Config 1: XDP prefilter (bpf/bpf_xdp.c:88-184)                         */
/* ===================================================================== */

static int xdp_one(or_dp *dp, const uint8_t *f, uint32_t len, uint8_t *nl)
{
    /* check_filters (:158-178): no room for ethhdr -> DROP */
    if (len < ETH_HLEN) return OR_XDP_DROP;
    uint16_t proto; memcpy(&proto, f + 12, 2);
    if (proto == 0x0008) {                     /* bpf_htons(ETH_P_IP) */
        /* check_v4 (:97-121) */
        if (len < ETH_HLEN + 20) return OR_XDP_DROP;
        uint32_t saddr, daddr; memcpy(&saddr, f + 26, 4); memcpy(&daddr, f + 30, 4);
        if (dp->v4_fix) {                      /* CIDR4_FILTER */
            or_lpm_v4_key k; k.prefixlen = 32; memcpy(k.addr, &saddr, 4);
            if (dp->v4_dyn) {                  /* CIDR4_LPM_PREFILTER */
                (*nl)++;
                if (or_map_lookup_ptr(dp->v4_dyn, &k)) return OR_XDP_DROP;
            }
            (*nl)++;
            if (or_map_lookup_ptr(dp->v4_fix, &k)) return OR_XDP_DROP;
        }
        /* check_v4_endpoint (:88-95) */
        return lookup_ip4_endpoint(dp, daddr, nl) ? OR_XDP_PASS : OR_XDP_DROP;
    } else if (proto == 0xDD86) {              /* bpf_htons(ETH_P_IPV6) */
        /* check_v6 (:132-156) */
        if (len < ETH_HLEN + 40) return OR_XDP_DROP;
        if (dp->v6_fix) {
            or_lpm_v6_key k; k.prefixlen = 128; memcpy(k.addr, f + 22, 16);
            if (dp->v6_dyn) {
                (*nl)++;
                if (or_map_lookup_ptr(dp->v6_dyn, &k)) return OR_XDP_DROP;
            }
            (*nl)++;
            if (or_map_lookup_ptr(dp->v6_fix, &k)) return OR_XDP_DROP;
        }
        return lookup_ip6_endpoint(dp, f + 38, nl) ? OR_XDP_PASS : OR_XDP_DROP;
    }
    return OR_XDP_PASS;
}

void or_xdp_prefilter(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                      uint32_t n, or_out *out)
{
    #pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < n; i++) {
        uint8_t nl = 0;
        uint32_t l = len[i] < stride ? len[i] : stride;  /* prefilter reads only the first 54 B */
        uint8_t v = xdp_one(dp, frames + (size_t)i * stride, l, &nl);
        if (out->xdp) out->xdp[i] = v;
        if (out->nl) out->nl[i] = nl;
        if (out->nu) out->nu[i] = 0;
        if (out->reason) out->reason[i] = 0;
    }
}

/* ===================================================================== */
/* Policy (bpf/lib/policy.h:46-200)                                      */
/* ===================================================================== */

static inline void ctr_add(or_policy_entry *p, uint32_t len)
{   /* __sync_fetch_and_add (policy.h:76-77, 88-89, 99-100) */
    __atomic_fetch_add(&p->packets, 1, __ATOMIC_RELAXED);
    __atomic_fetch_add(&p->bytes, (uint64_t)len, __ATOMIC_RELAXED);
}

/* __policy_can_access (policy.h:51-119); cb[CB_POLICY] is always 0 on this path
 * (policy_clear_mark at bpf_lxc.c:881, bpf_clear_cb at bpf_lxc.c:679). */
static int policy_can_access(or_map *map, uint32_t flags, uint32_t skb_len, uint32_t identity,
                             uint16_t dport, uint8_t proto, int dir, uint8_t *nl, uint8_t *nu)
{
    if (flags & OR_F_DROP_ALL) return OR_DROP_POLICY;
    or_policy_key key = { identity, dport, proto, (uint8_t)(!dir) };
    or_policy_entry *p;
    if (flags & OR_F_HAVE_L4_POLICY) {
        (*nl)++;
        p = or_map_lookup_ptr(map, &key);
        if (p) { ctr_add(p, skb_len); (*nu)++; return p->proxy_port; }
    }
    key.dport = 0; key.protocol = 0;
    (*nl)++;
    p = or_map_lookup_ptr(map, &key);
    if (p) { ctr_add(p, skb_len); (*nu)++; return OR_TC_ACT_OK; }
    if (flags & OR_F_HAVE_L4_POLICY) {
        key.sec_label = 0; key.dport = dport; key.protocol = proto;
        (*nl)++;
        p = or_map_lookup_ptr(map, &key);
        if (p) { ctr_add(p, skb_len); (*nu)++; return p->proxy_port; }
    }
    return OR_DROP_POLICY;
}

/* policy_can_access_ingress (policy.h:139-163) */
static int policy_can_access_ingress(or_map *map, uint32_t flags, uint32_t skb_len, uint32_t src,
                                     uint16_t dport, uint8_t proto, uint8_t *nl, uint8_t *nu)
{
    if (!(flags & OR_F_POLICY_INGRESS))
        return (flags & OR_F_DROP_ALL) ? OR_DROP_POLICY : OR_TC_ACT_OK;
    if (flags & OR_F_DROP_ALL) return OR_DROP_POLICY;
    int ret = policy_can_access(map, flags, skb_len, src, dport, proto, OR_CT_INGRESS, nl, nu);
    if (ret >= OR_TC_ACT_OK) return ret;
    return OR_DROP_POLICY;                      /* !IGNORE_DROP */
}

/* ===================================================================== */
/* Conntrack (bpf/lib/conntrack.h)                                        */
/* ===================================================================== */

#define CT_LIFETIME_TCP    21600
#define CT_LIFETIME_NONTCP 60
#define CT_SYN_TIMEOUT     60
#define CT_CLOSE_TIMEOUT   10
#define CT_REPORT_INTERVAL 5
#define TUPLE_F_OUT     0
#define TUPLE_F_IN      1
#define TUPLE_F_RELATED 2
#define TUPLE_F_SERVICE 4
#define ACTION_UNSPEC 0
#define ACTION_CREATE 1
#define ACTION_CLOSE  2
#define B_RX_CLOSING 0x1
#define B_TX_CLOSING 0x2
#define B_LB_LOOPBACK 0x8
#define B_SEEN_NON_SYN 0x10
#define TCPF_FIN 0x01   /* union tcp_flags.lower_bits: TCP flags byte (conntrack.h:74-86) */
#define TCPF_SYN 0x02
#define TCPF_RST 0x04

/* __ct_update_timeout (conntrack.h:103-161) */
static int ct_update_timeout_raw(or_ct_entry *e, uint32_t lifetime, int dir, uint8_t seen, uint32_t now)
{
    e->lifetime = now + lifetime;                        /* NEEDS_TIMEOUT (common.h:33) */
    uint8_t *acc = dir == OR_CT_INGRESS ? &e->rx_flags_seen : &e->tx_flags_seen;
    uint32_t *last = dir == OR_CT_INGRESS ? &e->last_rx_report : &e->last_tx_report;
    seen |= *acc;
    if (*last + CT_REPORT_INTERVAL < now || *acc != seen) {
        *last = now; *acc = seen;
        return 1;
    }
    return 0;
}

/* ct_update_timeout (conntrack.h:169-186) */
static int ct_update_timeout(or_ct_entry *e, int tcp, int dir, uint8_t seen, uint32_t now)
{
    uint32_t lifetime = CT_LIFETIME_NONTCP;
    if (tcp) {
        if (!(seen & TCPF_SYN)) e->bits |= B_SEEN_NON_SYN;
        lifetime = (e->bits & B_SEEN_NON_SYN) ? CT_LIFETIME_TCP : CT_SYN_TIMEOUT;
    }
    return ct_update_timeout_raw(e, lifetime, dir, seen, now);
}

static inline int ct_alive(const or_ct_entry *e)   /* conntrack.h:194-197 */
{
    return !(e->bits & B_RX_CLOSING) || !(e->bits & B_TX_CLOSING);
}

/* The accounting split (include/cilium_hip.h CV_F_ACCT_SPLIT): conntrack lookups and
 * writes count OR_ACCT_CT_UNIT in nl / nu, every other map lookup / write 1, so one run
 * gives the HBM-resident share of B(p).  Test infrastructure's knob, as the device's. */
static uint8_t or_ctu = 1;
void or_set_acct_split(int on) { or_ctu = on ? 32 : 1; }

/* __ct_lookup (conntrack.h:199-263) */
static int ct_lookup_one(or_map *map, const void *t, int action, int dir, or_ct_state *st,
                         int tcp, uint8_t seen, uint32_t skb_len, uint32_t now, uint32_t flags,
                         uint8_t *nl, uint8_t *nu, int *mon)
{
    *nl += or_ctu;
    or_ct_entry *e = or_map_lookup_ptr(map, t);
    if (!e) { *mon = 1; return OR_CT_NEW; }
    *nu += or_ctu;
    if (ct_alive(e)) *mon = ct_update_timeout(e, tcp, dir, seen, now);
    if (st) {
        st->rev_nat_index = e->rev_nat_index;
        st->loopback = (e->bits & B_LB_LOOPBACK) ? 1 : 0;
        st->slave = e->slave;
    }
    if (flags & OR_F_CT_ACCOUNTING) {
        if (dir == OR_CT_INGRESS) { e->rx_packets += 1; e->rx_bytes += skb_len; }
        else                      { e->tx_packets += 1; e->tx_bytes += skb_len; }
    }
    switch (action) {
    case ACTION_CREATE:
        if ((e->bits & B_RX_CLOSING) + ((e->bits & B_TX_CLOSING) >> 1) >= 1) {
            e->bits &= (uint16_t)~(B_RX_CLOSING | B_TX_CLOSING);
            *mon = ct_update_timeout(e, tcp, dir, seen, now);
        }
        break;
    case ACTION_CLOSE:
        if (dir == OR_CT_INGRESS) e->bits |= B_RX_CLOSING; else e->bits |= B_TX_CLOSING;
        *mon = 1;
        if (ct_alive(e)) break;
        ct_update_timeout_raw(e, CT_CLOSE_TIMEOUT, dir, seen, now);
        break;
    }
    return OR_CT_ESTABLISHED;
}

/* ipv4_ct_tuple_reverse (conntrack.h:414-431) */
static void ct_tuple_reverse4(or_ipv4_ct_tuple *t)
{
    uint32_t a = t->saddr; t->saddr = t->daddr; t->daddr = a;
    uint16_t p = t->sport; t->sport = t->dport; t->dport = p;
    if (t->flags & TUPLE_F_IN) t->flags &= (uint8_t)~TUPLE_F_IN; else t->flags |= TUPLE_F_IN;
}

/* ct_lookup4 (conntrack.h:442-562); *mon = the `monitor` result of the last
 * __ct_lookup (conntrack.h:199-263) it ran, untouched when none ran */
static int ct_lookup4m(or_map *ct, or_ipv4_ct_tuple *t, const uint8_t *f, uint32_t avail, uint32_t len,
                       int off, int dir, or_ct_state *st, uint32_t now, uint32_t flags, uint8_t *nl, uint8_t *nu,
                       int *mon)
{
    int action = ACTION_UNSPEC, r;
    int tcp = t->nexthdr == 6;
    uint8_t seen = 0;
    if (dir == OR_CT_INGRESS) t->flags = TUPLE_F_OUT;
    else if (dir == OR_CT_EGRESS) t->flags = TUPLE_F_IN;
    else if (dir == OR_CT_SERVICE) t->flags = TUPLE_F_SERVICE;
    else return OR_DROP_CT_INVALID_HDR;

    switch (t->nexthdr) {
    case 1: {                                         /* IPPROTO_ICMP */
        uint8_t type;
        r = ld(f, avail, len, off, 1, &type);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        t->sport = 0; t->dport = 0;
        switch (type) {
        case 3: case 11: case 12:                     /* DEST_UNREACH, TIME_EXCEEDED, PARAMETERPROB */
            t->flags |= TUPLE_F_RELATED; break;
        case 0:                                       /* ECHOREPLY: dport = ICMP_ECHO (raw 8) */
            t->dport = 8; break;
        case 8:                                       /* ECHO: sport = type, fall through */
            t->sport = type; /* fallthrough */
        default:
            action = ACTION_CREATE; break;
        }
        break;
    }
    case 6: {                                         /* IPPROTO_TCP */
        uint8_t fl[2];
        r = ld(f, avail, len, off + 12, 2, fl);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        seen = fl[1];
        action = (seen & (TCPF_RST | TCPF_FIN)) ? ACTION_CLOSE : ACTION_CREATE;
        r = ld(f, avail, len, off, 4, &t->dport);     /* loads dport then sport slots */
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        break;
    }
    case 17:                                          /* IPPROTO_UDP */
        r = ld(f, avail, len, off, 4, &t->dport);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        action = ACTION_CREATE;
        break;
    default:
        return OR_DROP_CT_UNKNOWN_PROTO;
    }

    int ret = ct_lookup_one(ct, t, action, dir, st, tcp, seen, len, now, flags, nl, nu, mon);
    if (ret != OR_CT_NEW)
        return (t->flags & TUPLE_F_RELATED) ? OR_CT_RELATED : OR_CT_REPLY;
    if (dir != OR_CT_SERVICE) {
        ct_tuple_reverse4(t);
        ret = ct_lookup_one(ct, t, action, dir, st, tcp, seen, len, now, flags, nl, nu, mon);
    }
    return ret;
}

int or_ct_lookup4(or_map *ct, or_ipv4_ct_tuple *t, const uint8_t *f, uint32_t avail, uint32_t len,
                  int off, int dir, or_ct_state *st, uint32_t now, uint32_t flags, uint8_t *nl, uint8_t *nu)
{
    int mon = 0;
    return ct_lookup4m(ct, t, f, avail, len, off, dir, st, now, flags, nl, nu, &mon);
}

/* ct_create4 (conntrack.h:663-744) */
int or_ct_create4(or_map *ct, or_ipv4_ct_tuple *t, uint32_t skb_len, int dir, const or_ct_state *st,
                  uint32_t now)
{
    or_ct_entry e; memset(&e, 0, sizeof(e));
    int tcp = t->nexthdr == 6;
    e.rev_nat_index = st->rev_nat_index;
    if (st->loopback) e.bits |= B_LB_LOOPBACK;
    e.slave = st->slave;
    ct_update_timeout(&e, tcp, dir, tcp ? TCPF_SYN : 0, now);
    if (dir == OR_CT_INGRESS) { e.rx_packets = 1; e.rx_bytes = skb_len; }
    else                      { e.tx_packets = 1; e.tx_bytes = skb_len; }
    e.src_sec_id = st->src_sec_id;
    if (or_map_update(ct, t, &e, 0) < 0) return OR_DROP_CT_CREATE_FAILED;
    if (st->addr) {
        uint8_t fl = t->flags; uint32_t sa = t->saddr, da = t->daddr;
        if (dir == OR_CT_INGRESS) t->saddr = st->addr; else t->daddr = st->addr;
        if (st->loopback) {
            t->flags = TUPLE_F_IN;
            if (dir == OR_CT_INGRESS) t->daddr = st->svc_addr; else t->saddr = st->svc_addr;
        }
        if (or_map_update(ct, t, &e, 0) < 0) return OR_DROP_CT_CREATE_FAILED;
        t->saddr = sa; t->daddr = da; t->flags = fl;
    }
    or_ipv4_ct_tuple it; memset(&it, 0, sizeof(it));
    it.daddr = t->daddr; it.saddr = t->saddr; it.nexthdr = 1;
    it.flags = t->flags | TUPLE_F_RELATED;
    e.bits |= B_SEEN_NON_SYN;
    if (or_map_update(ct, &it, &e, 0) < 0) return OR_DROP_CT_CREATE_FAILED;
    return 0;
}

/* ===================================================================== */
/* The skb: a writable copy of the frame record.  Loads and stores follow  */
/* skb_load_bytes / skb_store_bytes bounds (skb->len); bytes inside len    */
/* but beyond the record give OR_E_TRUNC.                                 */
/* ===================================================================== */

#define OR_SKB_MAX 256
typedef struct { uint8_t b[OR_SKB_MAX]; uint32_t avail, len; } or_skb;

static void skb_init(or_skb *s, const uint8_t *f, uint32_t stride, uint32_t len)
{
    uint32_t rec = stride < OR_SKB_MAX ? stride : OR_SKB_MAX;
    s->len = len;
    s->avail = len < rec ? len : rec;
    memcpy(s->b, f, s->avail);
}

static inline int sld(const or_skb *s, int off, uint32_t n, void *to) { return ld(s->b, s->avail, s->len, off, n, to); }

/* out->frames_out of packet i: the rewritten frame of a forwarded (TC_ACT_OK / REDIRECT,
 * not to the L7 proxy) IPv4 or IPv6 packet, else the input frame */
static void emit_frame(const or_out *out, uint32_t i, const uint8_t *in, uint32_t stride, const or_skb *s,
                       int32_t ret, uint16_t proxy)
{
    if (!out->frames_out) return;
    uint8_t *o = out->frames_out + (size_t)i * stride;
    memcpy(o, in, stride);
    const int ip = stride >= 14 && ((in[12] == 0x08 && in[13] == 0x00) || (in[12] == 0x86 && in[13] == 0xDD));
    if (ip && (ret == OR_TC_ACT_OK || ret == OR_TC_ACT_REDIRECT) && !proxy) memcpy(o, s->b, s->avail);
}

/* skb_store_bytes: 0, 1 (beyond len: the helper fails) or OR_E_TRUNC */
static inline int sst(or_skb *s, int off, uint32_t n, const void *from)
{
    if (off < 0 || (uint64_t)off + n > s->len) return 1;
    if ((uint64_t)off + n > s->avail) return OR_E_TRUNC;
    memcpy(s->b + off, from, n);
    return 0;
}

/* ---- checksum helpers of the packet rewrites -------------------------------
 * Third-party arithmetic: the Linux kernel's bpf_l3_csum_replace /
 * bpf_l4_csum_replace / bpf_csum_diff (net/core/filter.c) over csum_replace2/4,
 * csum_replace_by_diff, inet_proto_csum_replace{4,_by_diff} and csum_partial
 * (include/net/checksum.h, net/core/utils.c, arch/x86/lib/csum-partial_64.c) of the
 * container's kernel 6.18, for CHECKSUM_NONE skbs (BPF_PROG_TEST_RUN; fully
 * software-checksummed packets).  Pinned by tests/golden/csum_kernel.npz, produced
 * by running the helpers in the kernel (oracle/kernel_golden.py gen_csum).  Values
 * are in memory byte order (little-endian loads of network-order bytes). */
static inline uint32_t cs_add(uint32_t a, uint32_t b) { uint32_t r = a + b; return r + (r < b); }
static inline uint32_t cs_sub(uint32_t a, uint32_t b) { return cs_add(a, ~b); }
static inline uint16_t cs_fold(uint32_t x)
{
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return (uint16_t)~x;
}
static inline uint16_t cs16_add(uint16_t a, uint16_t b) { uint16_t r = (uint16_t)(a + b); return (uint16_t)(r + (r < b)); }

/* bpf_csum_diff(&from, 4, &to, 4, seed): the 16-bit folded sum of ~from, to, seed */
static uint32_t csum_diff4(uint32_t from, uint32_t to, uint32_t seed)
{
    uint64_t t = (uint64_t)seed + ((uint64_t)(~from) | ((uint64_t)to << 32));
    if (t < (uint64_t)seed) t++;                           /* addq + adcq $0 */
    uint64_t r = (t >> 32) + (t & 0xFFFFFFFFu);            /* add32_with_carry */
    uint32_t x = (uint32_t)r + (uint32_t)(r >> 32);
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}

/* bpf_csum_diff(from, 16, to, 16, seed) (the IPv6 address rewrites): the folded
 * ones-complement sum of seed, the complemented from words and the to words */
static uint32_t csum_diff16(const uint8_t *from, const uint8_t *to, uint32_t seed)
{
    uint64_t t = seed;
    for (int k = 0; k < 4; k++) {
        uint32_t f, g;
        memcpy(&f, from + 4 * k, 4); memcpy(&g, to + 4 * k, 4);
        t += (uint32_t)~f;
        t += g;
    }
    t = (t & 0xFFFFFFFFu) + (t >> 32);
    uint32_t x = (uint32_t)t + (uint32_t)(t >> 32);
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}

static inline uint16_t sum16_get(const or_skb *s, int off) { return (uint16_t)(s->b[off] | s->b[off + 1] << 8); }
static inline void sum16_put(or_skb *s, int off, uint16_t v) { s->b[off] = (uint8_t)v; s->b[off + 1] = (uint8_t)(v >> 8); }

/* the access check of both helpers: 0, OR_E_TRUNC (beyond the record), 1 (beyond the packet) */
static inline int csum_at(const or_skb *s, int off)
{
    if (off < 0 || (uint64_t)off + 2 > s->len) return 1;
    if ((uint64_t)off + 2 > s->avail) return OR_E_TRUNC;
    return 0;
}

/* bpf_l3_csum_replace: size 0 = by diff (to), 2 / 4 = replace from -> to */
static int l3_csum_replace(or_skb *s, int off, uint32_t from, uint32_t to, int size)
{
    int r = csum_at(s, off);
    if (r) return r;
    uint16_t c = sum16_get(s, off);
    if (size == 0) c = cs_fold(cs_add(to, ~(uint32_t)c));
    else if (size == 2) c = (uint16_t)~cs16_add(cs16_add((uint16_t)~c, (uint16_t)~(uint16_t)from), (uint16_t)to);
    else c = cs_fold(cs_add(cs_sub(~(uint32_t)c, from), to));
    sum16_put(s, off, c);
    return 0;
}

#define OR_F_PSEUDO_HDR 0x10u
#define OR_F_MARK_MANGLED_0 0x20u
/* bpf_l4_csum_replace (size in flags & 0xF; CHECKSUM_NONE: BPF_F_PSEUDO_HDR has no effect) */
static int l4_csum_replace(or_skb *s, int off, uint32_t from, uint32_t to, uint32_t flags)
{
    int r = csum_at(s, off);
    if (r) return r;
    uint16_t c = sum16_get(s, off);
    const int mm = (flags & OR_F_MARK_MANGLED_0) != 0;
    if (mm && !c) return 0;
    if ((flags & 0xF) == 0) c = cs_fold(cs_add(to, ~(uint32_t)c));
    else {
        if ((flags & 0xF) == 2) { from &= 0xFFFFu; to &= 0xFFFFu; }
        c = cs_fold(cs_add(cs_sub(~(uint32_t)c, from), to));
    }
    if (mm && !c) c = 0xFFFFu;                             /* CSUM_MANGLED_0 */
    sum16_put(s, off, c);
    return 0;
}

/* csum_l4_offset_and_flags (csum.h:44-64) */
static inline void l4_csum_off(uint8_t nexthdr, int *off, uint32_t *flags)
{
    *off = 0; *flags = 0;
    if (nexthdr == 6) *off = 16;
    else if (nexthdr == 17) { *off = 6; *flags = OR_F_MARK_MANGLED_0; }
    else if (nexthdr == 58) *off = 2;
}

static inline int csum_err(int r, int code) { return r == OR_E_TRUNC ? r : code; }

/* l4_modify_port (l4.h:50-60): L4 checksum (2-byte replace), then the port */
static int l4_modify_port(or_skb *s, int l4_off, int port_off, uint8_t nexthdr, uint16_t port, uint16_t old_port)
{
    int coff; uint32_t cfl;
    l4_csum_off(nexthdr, &coff, &cfl);
    int r = l4_csum_replace(s, l4_off + coff, old_port, port, cfl | 2);   /* csum_l4_replace: any offset */
    if (r) return csum_err(r, OR_DROP_CSUM_L4);
    r = sst(s, l4_off + port_off, 2, &port);
    return r ? csum_err(r, OR_DROP_WRITE_ERROR) : 0;
}

/* ipv4_l3 (l3.h:54-69): ipv4_dec_ttl (ipv4.h:30-43: TTL <= 1 -> DROP_INVALID, else the
 * 2-byte L3 checksum replace of the TTL and the new TTL), then the source MAC (when
 * given) and the destination MAC */
static int ipv4_l3(or_skb *skb, const uint8_t *smac, const uint8_t *dmac)
{
    uint8_t ttl = skb->b[22];
    if (ttl <= 1) return OR_DROP_INVALID;
    uint8_t nt = (uint8_t)(ttl - 1);
    int r = l3_csum_replace(skb, ETH_HLEN + 10, ttl, nt, 2);
    if (r) return csum_err(r, OR_DROP_CSUM_L3);
    skb->b[22] = nt;
    if (smac && sst(skb, 6, 6, smac)) return OR_DROP_WRITE_ERROR;
    if (sst(skb, 0, 6, dmac)) return OR_DROP_WRITE_ERROR;
    return OR_TC_ACT_OK;
}

_Static_assert(sizeof(or_endpoint_info) == 48, "struct endpoint_info");
/* ===================================================================== */
/* Ingress: from_netdev -> handle_ipv4 -> ipv4_policy                     */
/* ===================================================================== */

static inline int IS_ERR(int x) { return x < 0 || x == OR_TC_ACT_SHOT; }   /* common.h:231 */

typedef struct {
    uint8_t ct; uint16_t proxy; uint8_t nl, nu;
} pkt_state;

#define TCP_DPORT_OFF 2
#define TCP_SPORT_OFF 0

/* lb4_rev_nat / __lb4_rev_nat (lb.h:426-517): rewrites of the reverse translation;
 * checksums are not modelled (no verdict depends on them). */
static int lb4_rev_nat(or_dp *dp, or_skb *skb, int l4_off, const or_ct_state *st, or_ipv4_ct_tuple *t,
                       int tuple_saddr, uint8_t *nl)
{
    if (!dp->lb4_revnat) return 0;
    (*nl)++;
    or_lb4_reverse_nat *nat = or_map_lookup_ptr(dp->lb4_revnat, &st->rev_nat_index);
    if (!nat) return 0;
    int r;
    if (nat->port) {                                  /* reverse_map_l4_port (lb.h:222-252) */
        switch (t->nexthdr) {
        case 6: case 17: {
            uint16_t old;
            if ((r = sld(skb, l4_off + TCP_SPORT_OFF, 2, &old))) return r == OR_E_TRUNC ? r : OR_E_FAULT;
            if (nat->port != old && (r = l4_modify_port(skb, l4_off, TCP_SPORT_OFF, t->nexthdr, nat->port, old)))
                return r;
            break;
        }
        case 1: case 58: break;
        default: return OR_DROP_UNKNOWN_L4;
        }
    }
    uint32_t old_sip, new_sip = nat->address, sum = 0;
    if (tuple_saddr) { old_sip = t->saddr; t->saddr = new_sip; }
    else if ((r = sld(skb, ETH_HLEN + 12, 4, &old_sip))) return r == OR_E_TRUNC ? r : OR_E_FAULT;
    if (st->loopback) {
        uint32_t old_dip;
        if ((r = sld(skb, ETH_HLEN + 16, 4, &old_dip))) return r == OR_E_TRUNC ? r : OR_E_FAULT;
        if ((r = sst(skb, ETH_HLEN + 16, 4, &old_sip))) return r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR;
        sum = csum_diff4(old_dip, old_sip, 0);
        t->saddr = old_sip;
    }
    if ((r = sst(skb, ETH_HLEN + 12, 4, &new_sip))) return r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR;
    sum = csum_diff4(old_sip, new_sip, sum);          /* __lb4_rev_nat (lb.h:540-547) */
    if ((r = l3_csum_replace(skb, ETH_HLEN + 10, 0, sum, 0))) return csum_err(r, OR_DROP_CSUM_L3);
    int coff; uint32_t cfl;
    l4_csum_off(t->nexthdr, &coff, &cfl);
    if (coff && (r = l4_csum_replace(skb, l4_off + coff, 0, sum, cfl | OR_F_PSEUDO_HDR)))
        return csum_err(r, OR_DROP_CSUM_L4);
    return 0;
}

/* ipv4_policy (bpf/bpf_lxc.c:865-979) for endpoint `ep`, LXC_NAT46 off; its caller
 * tail_ipv4_policy (:981-993).  ifindex is skb->cb[CB_IFINDEX] set by
 * ipv4_local_delivery (l3.h:103-132).  Returns the program's final verdict
 * (TC_ACT_*; drops accounted as METRIC_INGRESS) or OR_E_TRUNC. */
static int ipv4_policy(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t ifindex, uint32_t src_label,
                       int skip_proxy, uint32_t now, pkt_state *ps, int32_t *reason)
{
    int ret;
    uint32_t len = skb->len;
    if (len < ETH_HLEN + 20) { ret = OR_DROP_INVALID; goto drop; }     /* revalidate_data */
    or_ipv4_ct_tuple t; memset(&t, 0, sizeof(t));
    or_ct_state st, st_new; memset(&st, 0, sizeof(st)); memset(&st_new, 0, sizeof(st_new));
    const uint8_t *f = skb->b;
    t.nexthdr = f[23];
    memcpy(&t.daddr, f + 30, 4); memcpy(&t.saddr, f + 26, 4);
    int l4_off = ETH_HLEN + (f[14] & 0x0F) * 4;
    int mon = 0;                                      /* bool monitor = false */
    ret = ct_lookup4m(ep->ct4, &t, skb->b, skb->avail, len, l4_off, OR_CT_INGRESS, &st, now, dp->flags,
                      &ps->nl, &ps->nu, &mon);
    if (ret < 0) goto drop;
    ps->ct = (uint8_t)ret;
    if (ret == OR_CT_REPLY && st.rev_nat_index && !st.loopback) {     /* :904-913 */
        int r2 = lb4_rev_nat(dp, skb, l4_off, &st, &t, 1, &ps->nl);
        if (IS_ERR(r2)) { ret = r2; goto drop; }
    }
    int verdict = policy_can_access_ingress(ep->policy, dp->flags, len, src_label, t.dport, t.nexthdr,
                                            &ps->nl, &ps->nu);
    if (ret != OR_CT_REPLY && ret != OR_CT_RELATED && verdict < 0) {
        if (ret == OR_CT_ESTABLISHED) {               /* ct_delete4 */
            if (or_map_delete(ep->ct4, &t) == 0) ps->nu += or_ctu;
        }
        ret = OR_DROP_POLICY;
        goto drop;
    }
    if (skip_proxy) verdict = 0;
    if (ret == OR_CT_NEW) {
        st_new.orig_dport = t.dport;
        st_new.src_sec_id = src_label;
        int r = or_ct_create4(ep->ct4, &t, len, OR_CT_INGRESS, &st_new, now);
        ps->nu += 2 * or_ctu;
        if (IS_ERR(r)) { ret = r; goto drop; }
    }
    if (verdict > 0 && (ret == OR_CT_NEW || ret == OR_CT_ESTABLISHED)) {
        /* ipv4_redirect_to_host_port (lib/lxc.h:97-142): rewrite + proxy-map insert
         * (L7 side effect, out of scope); the verdict redirects to HOST_IFINDEX. */
        notify_trace(dp, TRACE_TO_PROXY, len, ep->lxc_id, ep->seclabel, 0, 0, HOST_IFINDEX, (uint8_t)ret, mon);
        ps->proxy = (uint16_t)verdict;
        ifindex = HOST_IFINDEX;
    } else {
        update_metrics(dp, len, 1, 0);                /* send_trace_notify(TRACE_TO_LXC) */
        notify_trace(dp, TRACE_TO_LXC, len, ep->lxc_id, src_label, ep->seclabel, ep->lxc_id, ifindex,
                     (uint8_t)ret, mon);
    }
    if (ifindex) return OR_TC_ACT_REDIRECT;           /* redirect(ifindex, 0) */
    return OR_TC_ACT_OK;
drop:
    if (ret == OR_E_TRUNC) return ret;
    update_metrics(dp, len, 1, (uint8_t)(-ret));      /* tail_ipv4_policy: send_drop_notify */
    notify_drop(dp, ret, len, ep->lxc_id, src_label, ep->seclabel, ep->lxc_id, ifindex);
    if (reason) *reason = ret;
    return OR_TC_ACT_SHOT;
}

static int ipv6_policy(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t ifindex, uint32_t src_label,
                       int skip_proxy, uint32_t now, pkt_state *ps, int32_t *reason);

/* handle_policy (bpf_lxc.c:1003-1038): the cilium_policy[lxc_id] tail-call target;
 * DROP_ALL drops before any conntrack work; an IPv4 packet needs LXC_IPV4. */
static int handle_policy(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t ifindex, uint32_t src_label,
                         int skip_proxy, uint32_t now, pkt_state *ps, int32_t *reason)
{
    uint16_t proto = 0;
    if (skb->avail >= 14) memcpy(&proto, skb->b + 12, 2);
    int ret;
    if (dp->flags & OR_F_DROP_ALL) ret = OR_DROP_POLICY;
    else if (proto == 0xDD86) {
        if (ep->ct6) return ipv6_policy(dp, ep, skb, ifindex, src_label, skip_proxy, now, ps, reason);
        ret = OR_DROP_MISSED_TAIL_CALL;
    } else if (proto == 0x0008 && ep->ipv4) {
        return ipv4_policy(dp, ep, skb, ifindex, src_label, skip_proxy, now, ps, reason);
    } else ret = OR_DROP_UNKNOWN_L3;
    update_metrics(dp, skb->len, 1, (uint8_t)(-ret));   /* bpf_lxc.c:1032-1035 */
    notify_drop(dp, ret, skb->len, ep->lxc_id, src_label, ep->seclabel, ep->lxc_id, ifindex);
    if (reason) *reason = ret;
    return OR_TC_ACT_SHOT;
}

/* handle_ipv4 (bpf/bpf_netdev.c:357-453), ENCAP_IFINDEX paths (overlay) disabled,
 * reverse_proxy with an empty cilium_proxy4 map (L7 out of scope).  When the packet
 * reaches the endpoint, the tail-called policy program (handle_policy ->
 * tail_ipv4_policy, bpf_lxc.c:981-1038) runs and its return value is final:
 * *final = 1 and the return is TC_ACT_SHOT / TC_ACT_OK / TC_ACT_REDIRECT. */
static int handle_ipv4(or_dp *dp, or_skb *skb, uint32_t src_identity, int skip_proxy, uint32_t now,
                       uint32_t *out_identity, pkt_state *ps, int *final, int32_t *reason)
{
    *final = 0;
    uint32_t len = skb->len;
    const uint8_t *f = skb->b;
    if (len < ETH_HLEN + 20) return OR_DROP_INVALID;
    int l4_off = ETH_HLEN + (f[14] & 0x0F) * 4;
    uint32_t secctx = WORLD_ID;                        /* derive_ipv4_sec_ctx (:278-290) */
    uint8_t nexthdr = f[23];
    uint32_t saddr, daddr; memcpy(&saddr, f + 26, 4); memcpy(&daddr, f + 30, 4);
    if (src_identity < HEALTH_ID) {                    /* identity_is_reserved (policy.h:46-49) */
        or_remote_endpoint_info *info = ipcache_lookup4(dp, saddr, 32, &ps->nl);
        if (info && info->sec_label && info->sec_label != CLUSTER_ID && info->sec_label != HOST_ID)
            src_identity = info->sec_label;
    }
    *out_identity = src_identity;
    if (dp->flags & OR_F_FROM_HOST) {
        secctx = src_identity;
        if (nexthdr == 6 || nexthdr == 17) {           /* reverse_proxy (:293-354): port load */
            uint8_t p[4];
            int r = sld(skb, l4_off, 4, p);
            if (r == OR_E_TRUNC) return r;
            if (r) return OR_DROP_CT_INVALID_HDR;
        }
        sst(skb, 0, 6, dp->net_mac);                   /* rewrite_dmac_to_host (:156-169) */
    }
    or_endpoint_info *ep = lookup_ip4_endpoint(dp, daddr, &ps->nl);
    if (ep) {
        if (ep->flags & 1) return OR_TC_ACT_OK;        /* ENDPOINT_F_HOST */
        /* ipv4_local_delivery (l3.h:103-132): ipv4_l3 -> ipv4_dec_ttl, MACs */
        int rl3 = ipv4_l3(skb, ep->node_mac, ep->mac);
        if (rl3 != OR_TC_ACT_OK) return rl3;
        or_endpoint_prog *prog = find_ep(dp, ep->lxc_id);
        if (!prog) return OR_DROP_MISSED_TAIL_CALL;   /* tail_call(cilium_policy, lxc_id) missed */
        *final = 1;
        return handle_policy(dp, prog, skb, ep->ifindex, secctx, skip_proxy, now, ps, reason);
    }
    return OR_TC_ACT_OK;
}

static int handle_ipv6(or_dp *dp, or_skb *skb, uint32_t src_identity, int skip_proxy, uint32_t now,
                       uint32_t *out_identity, pkt_state *ps, int *final, int32_t *reason);

/* handle_identity_from_host (bpf_netdev.c:128-153) */
static uint32_t identity_from_mark(uint32_t mark, int *skip_proxy)
{
    uint32_t magic = mark & 0xF00;
    if (magic == 0xA00) { *skip_proxy = 1; return ((mark & 0xFF) << 16) | (mark >> 16); }
    if (magic == 0xB00) return ((mark & 0xFF) << 16) | (mark >> 16);
    if (magic == 0xC00) return HOST_ID;
    return WORLD_ID;
}

void or_netdev_ingress(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                       const uint32_t *mark, uint32_t n, uint32_t now, int with_prefilter, or_out *out)
{
    or_skb skb;
    for (uint32_t i = 0; i < n; i++) {
        skb_init(&skb, frames + (size_t)i * stride, stride, len[i]);
        uint32_t L = len[i];
        dp->cur_pkt = i;
        dp->cur_hash = 0;                              /* no skb hash input on this entry point */
        pkt_state ps = { OR_CT_NONE, 0, 0, 0 };
        uint8_t xv = OR_XDP_PASS;
        int32_t ret = OR_TC_ACT_OK, reason = 0;
        uint32_t ident = 0;
        if (with_prefilter) xv = (uint8_t)xdp_one(dp, skb.b, skb.avail, &ps.nl);
        if (xv == OR_XDP_PASS) {
            /* from_netdev (bpf_netdev.c:470-524) */
            uint32_t identity = 0; int skip_proxy = 0;
            if (dp->flags & OR_F_FROM_HOST) {
                const uint32_t magic = (mark ? mark[i] : 0) & 0xF00;   /* from_proxy: 0xA00 / 0xB00 */
                identity = identity_from_mark(mark ? mark[i] : 0, &skip_proxy);
                notify_trace(dp, magic == 0xA00 || magic == 0xB00 ? TRACE_FROM_PROXY : TRACE_FROM_HOST, L, 0,
                             identity, 0, 0, dp->ingress_ifindex, 0, 1);
            } else {
                notify_trace(dp, TRACE_FROM_STACK, L, 0, 0, 0, 0, dp->ingress_ifindex, 0, 1);
            }
            uint16_t proto = 0;
            if (skb.avail >= 14) memcpy(&proto, skb.b + 12, 2);      /* skb->protocol */
            ident = identity;
            if (proto == 0x0008 || proto == 0xDD86) {
                int final = 0;
                /* IPv4: tail_handle_ipv4 (:457-466); IPv6: handle_ipv6 inline (:495-503) */
                int r = proto == 0x0008 ? handle_ipv4(dp, &skb, identity, skip_proxy, now, &ident, &ps, &final, &reason)
                                        : handle_ipv6(dp, &skb, identity, skip_proxy, now, &ident, &ps, &final, &reason);
                if (r == OR_E_LDABS) ret = OR_TC_ACT_OK;         /* the program exited with 0 */
                else if (r == OR_E_TRUNC || r == OR_E_PUNT || final) ret = r;
                else if (IS_ERR(r)) {
                    update_metrics(dp, L, 1, (uint8_t)(-r));
                    notify_drop(dp, r, L, 0, 0, 0, 0, 0);        /* send_drop_notify_error */
                    reason = r;
                    ret = OR_TC_ACT_SHOT;
                } else ret = r;
            } else {
                ret = OR_TC_ACT_OK;                          /* unknown traffic to the stack (:518-521) */
            }
        }
        if (out->xdp) out->xdp[i] = xv;
        emit_frame(out, i, frames + (size_t)i * stride, stride, &skb, ret, ps.proxy);
        if (out->ret) out->ret[i] = ret;
        if (out->identity) out->identity[i] = ident;
        if (out->ct) out->ct[i] = ps.ct;
        if (out->proxy) out->proxy[i] = ps.proxy;
        if (out->nl) out->nl[i] = ps.nl;
        if (out->nu) out->nu[i] = ps.nu;
        if (out->reason) out->reason[i] = reason;
    }
}

/* ===================================================================== */
/* Config 2: stateless ingress verdict for one endpoint                   */
/* ===================================================================== */

void or_policy_ingress(or_dp *dp, uint32_t ep_index, const uint8_t *frames, uint32_t stride,
                       const uint32_t *len, const uint32_t *mark, uint32_t n, or_out *out)
{
    or_endpoint_prog *ep = &dp->ep[ep_index];
    #pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *f = frames + (size_t)i * stride;
        uint32_t L = len[i], avail = L < stride ? L : stride;
        pkt_state ps = { OR_CT_NONE, 0, 0, 0 };
        int skip_proxy = 0;
        uint32_t identity = 0;
        int32_t ret;
        if (dp->flags & OR_F_FROM_HOST) identity = identity_from_mark(mark ? mark[i] : 0, &skip_proxy);
        uint16_t proto = 0;
        if (avail >= 14) memcpy(&proto, f + 12, 2);
        if (proto != 0x0008) {
            ret = OR_DROP_UNKNOWN_L3;
        } else if (L < ETH_HLEN + 20) {
            ret = OR_DROP_INVALID;
        } else {
            uint32_t saddr; memcpy(&saddr, f + 26, 4);
            if (identity < HEALTH_ID) {                       /* bpf_netdev.c:375-398 */
                or_remote_endpoint_info *info = ipcache_lookup4(dp, saddr, 32, &ps.nl);
                if (info && info->sec_label && info->sec_label != CLUSTER_ID && info->sec_label != HOST_ID)
                    identity = info->sec_label;
            }
            /* L4 key as ct_lookup4 (conntrack.h:471-530) leaves it after the reverse
             * (forward-direction) lookup of a NEW flow. */
            or_ipv4_ct_tuple t; memset(&t, 0, sizeof(t));
            t.nexthdr = f[23];
            int off = ETH_HLEN + (f[14] & 0x0F) * 4, r = 0;
            ret = 0;
            switch (t.nexthdr) {
            case 1: {
                uint8_t type;
                r = ld(f, avail, L, off, 1, &type);
                if (r == OR_E_TRUNC) { ret = r; break; }
                if (r) { ret = OR_DROP_CT_INVALID_HDR; break; }
                t.sport = 0; t.dport = 0;
                if (type == 0) t.dport = 8; else if (type == 8) t.sport = type;
                break;
            }
            case 6: {
                uint8_t fl[2];
                r = ld(f, avail, L, off + 12, 2, fl);
                if (!r) r = ld(f, avail, L, off, 4, &t.dport);
                if (r == OR_E_TRUNC) { ret = r; break; }
                if (r) { ret = OR_DROP_CT_INVALID_HDR; break; }
                break;
            }
            case 17:
                r = ld(f, avail, L, off, 4, &t.dport);
                if (r == OR_E_TRUNC) { ret = r; break; }
                if (r) { ret = OR_DROP_CT_INVALID_HDR; break; }
                break;
            default:
                ret = OR_DROP_CT_UNKNOWN_PROTO;
            }
            if (ret == 0) {
                uint16_t p = t.sport; t.sport = t.dport; t.dport = p;   /* ipv4_ct_tuple_reverse */
                int v = policy_can_access_ingress(ep->policy, dp->flags, L, identity, t.dport, t.nexthdr,
                                                  &ps.nl, &ps.nu);
                if (v < 0) ret = OR_DROP_POLICY;
                else { ret = v; if (!skip_proxy && v > 0) ps.proxy = (uint16_t)v; }
                if (skip_proxy && v > 0) ret = 0;
            }
        }
        if (ret < 0 && ret != OR_E_TRUNC) update_metrics(dp, L, 1, (uint8_t)(-ret));
        if (out->ret) out->ret[i] = ret;
        if (out->identity) out->identity[i] = identity;
        if (out->proxy) out->proxy[i] = ps.proxy;
        if (out->ct) out->ct[i] = OR_CT_NONE;
        if (out->nl) out->nl[i] = ps.nl;
        if (out->nu) out->nu[i] = ps.nu;
        if (out->reason) out->reason[i] = (ret < 0 && ret != OR_E_TRUNC) ? ret : 0;
    }
}

/* ===================================================================== */
/* Load balancer lookup (bpf/lib/lb.h:604-635), LB_L4 and LB_L3 on        */
/* ===================================================================== */

const or_lb4_service *or_lb4_lookup_service(or_map *svc_map, or_lb4_key *key, uint8_t *nl)
{
    if (key->dport) {
        (*nl)++;
        or_lb4_service *s = or_map_lookup_ptr(svc_map, key);
        if (s && s->count != 0) return s;
        key->dport = 0;
    }
    (*nl)++;
    or_lb4_service *s = or_map_lookup_ptr(svc_map, key);
    if (s && s->count != 0) return s;
    return NULL;
}

/* lb4_lookup_slave (lb.h:637-651) */
static or_lb4_service *lb4_lookup_slave(or_map *m, or_lb4_key *key, uint16_t slave, uint8_t *nl)
{
    key->slave = slave;
    (*nl)++;
    return or_map_lookup_ptr(m, key);
}

/* lb4_select_slave / lb6_select_slave (lb.h:158-190, the WRR branch is #if 0):
 * slave 0 is the master, so (hash % count) + 1; hash = get_hash_recalc(), an input */
static inline uint16_t lb_select_slave(uint32_t hash, uint16_t count) { return (uint16_t)(hash % count + 1); }

/* lb6_lookup_service (lb.h:351-380) with LB_L4 and LB_L3 (pkg/endpoint/bpf.go:193-194) */
static or_lb6_service *lb6_lookup_service(or_map *m, or_lb6_key *key, uint8_t *nl)
{
    or_lb6_service *svc;
    if (!m) return NULL;
    if (key->dport) {
        (*nl)++;
        svc = or_map_lookup_ptr(m, key);
        if (svc && svc->count != 0) return svc;
        key->dport = 0;
    }
    (*nl)++;
    svc = or_map_lookup_ptr(m, key);
    if (svc && svc->count != 0) return svc;
    return NULL;
}

/* lb6_lookup_slave (lb.h:382-396) */
static or_lb6_service *lb6_lookup_slave(or_map *m, or_lb6_key *key, uint16_t slave, uint8_t *nl)
{
    key->slave = slave;
    (*nl)++;
    return or_map_lookup_ptr(m, key);
}

/* ct_update4_slave / ct_update6_slave (conntrack.h:572-586, 649-661) */
static void ct_update_slave(or_map *map, const void *t, const or_ct_state *st, uint8_t *nl, uint8_t *nu)
{
    *nl += or_ctu;
    or_ct_entry *e = or_map_lookup_ptr(map, t);
    if (!e) return;
    e->slave = st->slave;
    *nu += or_ctu;
}

/* extract_l4_port (lb.h:192-216): TCP/UDP dport; ICMP/ICMPv6 none; else DROP_UNKNOWN_L4 */
static int extract_l4_port(const or_skb *skb, uint8_t nexthdr, int l4_off, uint16_t *port)
{
    switch (nexthdr) {
    case 6: case 17: {
        int r = sld(skb, l4_off + TCP_DPORT_OFF, 2, port);   /* l4_load_port (l4.h:62-65) */
        if (r) return r == OR_E_TRUNC ? r : OR_E_FAULT;
        return 0;
    }
    case 58: case 1: return 0;
    default: return OR_DROP_UNKNOWN_L4;
    }
}

/* lb4_local (lb.h:700-775) + lb4_xlate (:653-697) */
static int lb4_local(or_dp *dp, or_map *ct, or_skb *skb, int l4_off, or_lb4_key *key, or_ipv4_ct_tuple *t,
                     or_lb4_service *svc, or_ct_state *st, uint32_t saddr, uint32_t hash, uint32_t now, pkt_state *ps)
{
    uint8_t flags = t->flags;
    uint32_t new_saddr = 0, new_daddr;
    int ret = or_ct_lookup4(ct, t, skb->b, skb->avail, skb->len, l4_off, OR_CT_SERVICE, st, now, dp->flags,
                            &ps->nl, &ps->nu);
    if (ret == OR_E_TRUNC) return ret;
    switch (ret) {
    case OR_CT_NEW:
        st->slave = lb_select_slave(hash, svc->count);
        ret = or_ct_create4(ct, t, skb->len, OR_CT_SERVICE, st, now);
        ps->nu += 2 * or_ctu;
        if (IS_ERR(ret)) { t->flags = flags; return OR_DROP_NO_SERVICE; }
        break;
    case OR_CT_ESTABLISHED: case OR_CT_RELATED: case OR_CT_REPLY:
        break;
    default:
        t->flags = flags;
        return OR_DROP_NO_SERVICE;
    }
    if (!(svc = lb4_lookup_slave(dp->lb4_services, key, st->slave, &ps->nl))) {
        if (!(svc = (or_lb4_service *)or_lb4_lookup_service(dp->lb4_services, key, &ps->nl))) {
            t->flags = flags;
            return OR_DROP_NO_SERVICE;
        }
        st->slave = lb_select_slave(hash, svc->count);
        ct_update_slave(ct, t, st, &ps->nl, &ps->nu);
    }
    t->flags = flags;
    st->rev_nat_index = svc->rev_nat_index;
    st->addr = new_daddr = svc->target;
    if (saddr == svc->target) {                       /* !DISABLE_LOOPBACK_LB (:753-767) */
        new_saddr = dp->v4_loopback;
        st->loopback = 1;
        st->addr = new_saddr;
        st->svc_addr = saddr;
    }
    if (!st->loopback) t->daddr = svc->target;
    /* lb4_xlate (lb.h:653-697): addresses, their checksum diff into the L3 and (pseudo
     * header) L4 checksums, then the service port */
    int r = sst(skb, ETH_HLEN + 16, 4, &new_daddr);
    if (r) return r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR;
    uint32_t sum = csum_diff4(key->address, new_daddr, 0);
    if (new_saddr) {
        r = sst(skb, ETH_HLEN + 12, 4, &new_saddr);
        if (r) return r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR;
        sum = csum_diff4(saddr, new_saddr, sum);
    }
    if ((r = l3_csum_replace(skb, ETH_HLEN + 10, 0, sum, 0))) return csum_err(r, OR_DROP_CSUM_L3);
    int coff; uint32_t cfl;
    l4_csum_off(t->nexthdr, &coff, &cfl);
    if (coff && (r = l4_csum_replace(skb, l4_off + coff, 0, sum, cfl | OR_F_PSEUDO_HDR)))
        return csum_err(r, OR_DROP_CSUM_L4);
    if (svc->port && key->dport != svc->port && (t->nexthdr == 6 || t->nexthdr == 17)) {
        r = l4_modify_port(skb, l4_off, TCP_DPORT_OFF, t->nexthdr, svc->port, key->dport);
        if (r) return r;
    }
    return OR_TC_ACT_OK;
}

/* policy_can_egress (policy.h:181-200) with POLICY_EGRESS && LXC_ID */
static int policy_can_egress(or_map *map, uint32_t flags, uint32_t len, uint32_t identity, uint16_t dport,
                             uint8_t proto, uint8_t *nl, uint8_t *nu)
{
    if (!(flags & OR_F_POLICY_EGRESS)) return (flags & OR_F_DROP_ALL) ? OR_DROP_POLICY : OR_TC_ACT_OK;
    if (flags & OR_F_DROP_ALL) return OR_DROP_POLICY;
    int ret = policy_can_access(map, flags, len, identity, dport, proto, OR_CT_EGRESS, nl, nu);
    if (ret >= 0) return ret;
    return OR_DROP_POLICY;
}

/* handle_ipv4_from_lxc (bpf_lxc.c:402-649) of endpoint `ep`, direct routing (no
 * ENCAP_IFINDEX), LXC_NAT46 off.  A local destination gets the tail call into its
 * policy program: *final = 1 and the return is that program's verdict. */
static int handle_ipv4_from_lxc(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t hash, uint32_t now,
                                uint32_t *dst_id, pkt_state *ps, int *final, int32_t *reason)
{
    or_ipv4_ct_tuple t; memset(&t, 0, sizeof(t));
    or_ct_state st_new, st; memset(&st_new, 0, sizeof(st_new)); memset(&st, 0, sizeof(st));
    or_lb4_key key; memset(&key, 0, sizeof(key));
    uint32_t len = skb->len;
    uint8_t *f = skb->b;
    int ret, verdict;
    *final = 0;
    if (len < ETH_HLEN + 20) return OR_DROP_INVALID;               /* revalidate_data */
    t.nexthdr = f[23];
    if (memcmp(f + 6, ep->mac, 6)) return OR_DROP_INVALID_SMAC;    /* is_valid_lxc_src_mac (lxc.h:31-37) */
    if (memcmp(f + 0, ep->node_mac, 6)) return OR_DROP_INVALID_DMAC;  /* is_valid_gw_dst_mac (:69-75) */
    uint32_t saddr; memcpy(&saddr, f + 26, 4);
    if (saddr != ep->ipv4) return OR_DROP_INVALID_SIP;             /* is_valid_lxc_src_ipv4 (:54-61) */
    memcpy(&t.daddr, f + 30, 4);
    t.saddr = saddr;
    int l4_off = ETH_HLEN + (f[14] & 0x0F) * 4;
    /* lb4_extract_key (lb.h:519-541): key.address = daddr (CT_EGRESS) */
    key.address = t.daddr;
    ret = extract_l4_port(skb, t.nexthdr, l4_off, &key.dport);
    if (ret == OR_E_TRUNC) return ret;
    if (IS_ERR(ret)) {
        if (ret != OR_DROP_UNKNOWN_L4) return ret;
    } else {
        st_new.orig_dport = key.dport;
        or_lb4_service *svc = (or_lb4_service *)(dp->lb4_services ? or_lb4_lookup_service(dp->lb4_services, &key, &ps->nl) : NULL);
        if (svc) {
            ret = lb4_local(dp, ep->ct4, skb, l4_off, &key, &t, svc, &st_new, saddr, hash, now, ps);
            if (ret == OR_E_TRUNC || IS_ERR(ret)) return ret;
        }
    }
    uint32_t orig_dip = t.daddr;                                    /* skip_service_lookup: */
    int mon = 0;                                      /* bool monitor = false (lb4_local's is its own) */
    ret = ct_lookup4m(ep->ct4, &t, skb->b, skb->avail, len, l4_off, OR_CT_EGRESS, &st, now, dp->flags,
                      &ps->nl, &ps->nu, &mon);
    if (ret < 0) return ret;
    ps->ct = (uint8_t)ret;
    /* destination category (:482-494) */
    uint32_t dst = WORLD_ID;
    or_remote_endpoint_info *info = ipcache_lookup4(dp, orig_dip, 32, &ps->nl);
    if (info && info->sec_label) dst = info->sec_label;
    else if ((orig_dip & dp->v4_cluster_mask) == dp->v4_cluster_range) dst = CLUSTER_ID;
    *dst_id = dst;
    verdict = policy_can_egress(ep->policy, dp->flags, len, dst, t.dport, t.nexthdr, &ps->nl, &ps->nu);
    if (ret != OR_CT_REPLY && ret != OR_CT_RELATED && verdict < 0) {
        if (ret == OR_CT_ESTABLISHED) {                             /* ct_delete4 */
            if (or_map_delete(ep->ct4, &t) == 0) ps->nu += or_ctu;
        }
        return verdict;
    }
    switch (ret) {
    case OR_CT_NEW: {
        st_new.src_sec_id = ep->seclabel;
        int nat = st_new.addr != 0;
        int r = or_ct_create4(ep->ct4, &t, len, OR_CT_EGRESS, &st_new, now);
        ps->nu += (nat ? 3 : 2) * or_ctu;
        if (IS_ERR(r)) return r;
        break;
    }
    case OR_CT_ESTABLISHED:
        break;
    case OR_CT_RELATED: case OR_CT_REPLY:
        if (st.rev_nat_index) {
            int r = lb4_rev_nat(dp, skb, l4_off, &st, &t, 0, &ps->nl);
            if (r == OR_E_TRUNC || IS_ERR(r)) return r;
        }
        break;
    default:
        return OR_DROP_POLICY;
    }
    if (verdict > 0) {                                              /* redirect_to_proxy */
        /* ipv4_redirect_to_host_port: dport := proxy port, daddr := IPV4_GATEWAY,
         * proxy-map insert (L7 side effect, out of scope) */
        notify_trace(dp, TRACE_TO_PROXY, len, ep->lxc_id, ep->seclabel, 0, 0, HOST_IFINDEX, ps->ct, mon);
        ps->proxy = (uint16_t)verdict;
        int r = ipv4_l3(skb, ep->node_mac, dp->host_mac);
        if (r != OR_TC_ACT_OK) return r;
        return OR_TC_ACT_REDIRECT;                                  /* redirect(HOST_IFINDEX) */
    }
    uint32_t daddr; memcpy(&daddr, skb->b + 30, 4);                 /* after the L4/L3 rewrites */
    or_endpoint_info *dep = lookup_ip4_endpoint(dp, daddr, &ps->nl);
    if (dep) {
        /* to_host: ipv4_l3(NODE_MAC, HOST_IFINDEX_MAC); local: ipv4_local_delivery (l3.h:
         * 103-132) ipv4_l3(endpoint_info.node_mac, endpoint_info.mac) */
        int r = (dep->flags & 1) ? ipv4_l3(skb, ep->node_mac, dp->host_mac)
                                 : ipv4_l3(skb, dep->node_mac, dep->mac);
        if (r != OR_TC_ACT_OK) return r;
        update_metrics(dp, len, 2, 0);            /* to_host: TRACE_TO_HOST / ipv4_local_delivery */
        if (dep->flags & 1) {                                       /* ENDPOINT_F_HOST: redirect(HOST_IFINDEX) */
            notify_trace(dp, TRACE_TO_HOST, len, ep->lxc_id, ep->seclabel, HOST_ID, 0, HOST_IFINDEX, ps->ct, mon);
            return OR_TC_ACT_REDIRECT;
        }
        or_endpoint_prog *prog = find_ep(dp, dep->lxc_id);
        if (!prog) return OR_DROP_MISSED_TAIL_CALL;
        *final = 1;                                                 /* handle_policy -> tail_ipv4_policy */
        if (dp->split) {                                            /* (or_lxc_egress_split) */
            dp->pend_ep = (int32_t)(prog - dp->ep);
            dp->pend_ifindex = dep->ifindex;
            dp->pend_label = ep->seclabel;
            return OR_E_DEFER;
        }
        uint8_t ct_egress = ps->ct;                                 /* out.ct reports the egress CT result */
        r = handle_policy(dp, prog, skb, dep->ifindex, ep->seclabel, 0, now, ps, reason);
        ps->ct = ct_egress;
        return r;
    }
    int r = ipv4_l3(skb, NULL, ep->node_mac);                      /* pass_to_stack */
    if (r != OR_TC_ACT_OK) return r;
    update_metrics(dp, len, 2, 0);                                  /* TRACE_TO_STACK */
    notify_trace(dp, TRACE_TO_STACK, len, ep->lxc_id, ep->seclabel, dst, 0, 0, ps->ct, mon);
    return OR_TC_ACT_OK;
}

/* ===================================================================== */
/* IPv6                                                                   */
/* ===================================================================== */

/* ipv6_hdrlen (ipv6.h:61-98); the AUTH length is chosen by the type of the header
 * that FOLLOWS (nh is updated first), as the reference does */
static int ipv6_hdrlen(const or_skb *skb, int l3_off, uint8_t *nexthdr)
{
    int len = 40;
    uint8_t nh = *nexthdr;
    for (int i = 0; i < 4; i++) {
        switch (nh) {
        case 59: return OR_DROP_INVALID_EXTHDR;
        case 44: return OR_DROP_FRAG_NOSUPPORT;
        case 0: case 43: case 51: case 60: {
            uint8_t opt[2];
            int r = sld(skb, l3_off + len, 2, opt);
            if (r == OR_E_TRUNC) return r;
            if (r) return OR_DROP_INVALID;
            nh = opt[0];
            if (nh == 51) len += (opt[1] + 2) << 2;
            else len += (opt[1] + 1) << 3;
            break;
        }
        default:
            *nexthdr = nh;
            return len;
        }
    }
    return OR_DROP_INVALID_EXTHDR;
}

/* ipv6_ct_tuple_reverse (conntrack.h:265-285) */
static void ct_tuple_reverse6(or_ipv6_ct_tuple *t)
{
    uint8_t a[16]; memcpy(a, t->saddr, 16); memcpy(t->saddr, t->daddr, 16); memcpy(t->daddr, a, 16);
    uint16_t p = t->sport; t->sport = t->dport; t->dport = p;
    if (t->flags & TUPLE_F_IN) t->flags &= (uint8_t)~TUPLE_F_IN; else t->flags |= TUPLE_F_IN;
}

/* ct_lookup6 (conntrack.h:288-412) */
static int ct_lookup6(or_map *ct, or_ipv6_ct_tuple *t, const or_skb *skb, int off, int dir, or_ct_state *st,
                      uint32_t now, uint32_t flags, uint8_t *nl, uint8_t *nu, int *mon)
{
    int action = ACTION_UNSPEC, r;
    int tcp = t->nexthdr == 6;
    uint8_t seen = 0;
    if (dir == OR_CT_INGRESS) t->flags = TUPLE_F_OUT;
    else if (dir == OR_CT_EGRESS) t->flags = TUPLE_F_IN;
    else if (dir == OR_CT_SERVICE) t->flags = TUPLE_F_SERVICE;
    else return OR_DROP_CT_INVALID_HDR;
    switch (t->nexthdr) {
    case 58: {                                        /* IPPROTO_ICMPV6 */
        uint8_t type;
        r = sld(skb, off, 1, &type);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        t->sport = 0; t->dport = 0;
        switch (type) {
        case 1: case 2: case 3: case 4:               /* DEST_UNREACH, PKT_TOOBIG, TIME_EXCEED, PARAMPROB */
            t->flags |= TUPLE_F_RELATED; break;
        case 129:                                     /* ECHO_REPLY: dport = ICMPV6_ECHO_REQUEST (raw 128) */
            t->dport = 128; break;
        case 128:                                     /* ECHO_REQUEST */
            t->sport = type; /* fallthrough */
        default:
            action = ACTION_CREATE; break;
        }
        break;
    }
    case 6: {
        uint8_t fl[2];
        r = sld(skb, off + 12, 2, fl);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        seen = fl[1];
        action = (seen & (TCPF_RST | TCPF_FIN)) ? ACTION_CLOSE : ACTION_CREATE;
        r = sld(skb, off, 4, &t->dport);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        break;
    }
    case 17:
        r = sld(skb, off, 4, &t->dport);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_DROP_CT_INVALID_HDR;
        action = ACTION_CREATE;
        break;
    default:
        return OR_DROP_CT_UNKNOWN_PROTO;
    }
    int ret = ct_lookup_one(ct, t, action, dir, st, tcp, seen, skb->len, now, flags, nl, nu, mon);
    if (ret != OR_CT_NEW) return (t->flags & TUPLE_F_RELATED) ? OR_CT_RELATED : OR_CT_REPLY;
    if (dir != OR_CT_SERVICE) {
        ct_tuple_reverse6(t);
        ret = ct_lookup_one(ct, t, action, dir, st, tcp, seen, skb->len, now, flags, nl, nu, mon);
    }
    return ret;
}

/* ct_create6 (conntrack.h:588-639) */
static int ct_create6(or_map *ct, const or_ipv6_ct_tuple *t, uint32_t skb_len, int dir, const or_ct_state *st,
                      uint32_t now)
{
    or_ct_entry e; memset(&e, 0, sizeof(e));
    int tcp = t->nexthdr == 6;
    e.rev_nat_index = st->rev_nat_index;
    if (st->loopback) e.bits |= B_LB_LOOPBACK;
    e.slave = st->slave;
    ct_update_timeout(&e, tcp, dir, tcp ? TCPF_SYN : 0, now);
    if (dir == OR_CT_INGRESS) { e.rx_packets = 1; e.rx_bytes = skb_len; }
    else                      { e.tx_packets = 1; e.tx_bytes = skb_len; }
    e.src_sec_id = st->src_sec_id;
    if (or_map_update(ct, t, &e, 0) < 0) return OR_DROP_CT_CREATE_FAILED;
    or_ipv6_ct_tuple it; memset(&it, 0, sizeof(it));
    it.nexthdr = 58;
    it.flags = t->flags | TUPLE_F_RELATED;
    e.bits |= B_SEEN_NON_SYN;
    memcpy(it.daddr, t->daddr, 16); memcpy(it.saddr, t->saddr, 16);
    if (or_map_update(ct, &it, &e, 0) < 0) return OR_DROP_CT_CREATE_FAILED;
    return 0;
}

/* lb6_rev_nat / __lb6_rev_nat (lb.h:254-315), flags = 0 on every caller here:
 * rewrites the source address (and port) of the packet, then the L4 checksum by
 * the 16-byte diff (csum_l4_replace at the nexthdr's offset, 0 for unknown L4) */
static int lb6_rev_nat(or_dp *dp, or_skb *skb, int l4_off, uint16_t index, const or_ipv6_ct_tuple *t, uint8_t *nl)
{
    if (!dp->lb6_revnat) return 0;
    (*nl)++;
    or_lb6_reverse_nat *nat = or_map_lookup_ptr(dp->lb6_revnat, &index);
    if (!nat) return 0;
    int r;
    if (nat->port) {
        switch (t->nexthdr) {
        case 6: case 17: {
            uint16_t old;
            if ((r = sld(skb, l4_off + TCP_SPORT_OFF, 2, &old))) return r == OR_E_TRUNC ? r : OR_E_FAULT;
            if (nat->port != old && (r = l4_modify_port(skb, l4_off, TCP_SPORT_OFF, t->nexthdr, nat->port, old)))
                return r;
            break;
        }
        case 1: case 58: break;
        default: return OR_DROP_UNKNOWN_L4;
        }
    }
    uint8_t old[16];
    if ((r = sld(skb, ETH_HLEN + 8, 16, old))) return r == OR_E_TRUNC ? r : OR_DROP_INVALID;   /* ipv6_load_saddr */
    if ((r = sst(skb, ETH_HLEN + 8, 16, nat->address))) return r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR;
    uint32_t sum = csum_diff16(old, nat->address, 0);
    int coff; uint32_t cfl;
    l4_csum_off(t->nexthdr, &coff, &cfl);
    if ((r = l4_csum_replace(skb, l4_off + coff, 0, sum, cfl | OR_F_PSEUDO_HDR))) return csum_err(r, OR_DROP_CSUM_L4);
    return 0;
}

/* lb6_local (lb.h:426-483) + lb6_xlate (:386-424) */
static int lb6_local(or_dp *dp, or_map *ct, or_skb *skb, int l4_off, or_lb6_key *key, or_ipv6_ct_tuple *t,
                     or_lb6_service *svc, or_ct_state *st, uint32_t hash, uint32_t now, pkt_state *ps)
{
    uint8_t flags = t->flags;
    int mon = 0;                                      /* "Deliberately ignored" (lb.h:431) */
    int ret = ct_lookup6(ct, t, skb, l4_off, OR_CT_SERVICE, st, now, dp->flags, &ps->nl, &ps->nu, &mon);
    if (ret == OR_E_TRUNC) return ret;
    switch (ret) {
    case OR_CT_NEW:
        st->slave = lb_select_slave(hash, svc->count);
        ret = ct_create6(ct, t, skb->len, OR_CT_SERVICE, st, now);
        ps->nu += 2 * or_ctu;
        if (IS_ERR(ret)) { t->flags = flags; return OR_DROP_NO_SERVICE; }
        break;
    case OR_CT_ESTABLISHED: case OR_CT_RELATED: case OR_CT_REPLY:
        break;
    default:
        t->flags = flags;
        return OR_DROP_NO_SERVICE;
    }
    if (!(svc = lb6_lookup_slave(dp->lb6_services, key, st->slave, &ps->nl))) {
        if (!(svc = lb6_lookup_service(dp->lb6_services, key, &ps->nl))) {
            t->flags = flags;
            return OR_DROP_NO_SERVICE;
        }
        st->slave = lb_select_slave(hash, svc->count);
        ct_update_slave(ct, t, st, &ps->nl, &ps->nu);
    }
    t->flags = flags;
    memcpy(t->daddr, svc->target, 16);
    st->rev_nat_index = svc->rev_nat_index;
    int r = sst(skb, ETH_HLEN + 24, 16, svc->target);              /* lb6_xlate: ipv6_store_daddr */
    if (r == OR_E_TRUNC) return r;
    int coff; uint32_t cfl;                                         /* csum_off of lb6_extract_key */
    l4_csum_off(t->nexthdr, &coff, &cfl);
    r = l4_csum_replace(skb, l4_off + coff, 0, csum_diff16(key->address, svc->target, 0), cfl | OR_F_PSEUDO_HDR);
    if (r) return csum_err(r, OR_DROP_CSUM_L4);
    if (svc->port && key->dport != svc->port && (t->nexthdr == 6 || t->nexthdr == 17)) {
        r = l4_modify_port(skb, l4_off, TCP_DPORT_OFF, t->nexthdr, svc->port, key->dport);
        if (r) return r;
    }
    return OR_TC_ACT_OK;
}

/* ipv6_l3 (l3.h:30-51): ipv6_dec_hoplimit (ipv6.h:178-193; hop limit <= 1 ->
 * icmp6_send_time_exceeded tail call), then the source MAC (when given) and the
 * destination MAC */
static int ipv6_l3(or_skb *skb, const uint8_t *smac, const uint8_t *dmac)
{
    uint8_t hl = skb->b[21];
    if (hl <= 1) return OR_E_PUNT;
    skb->b[21] = (uint8_t)(hl - 1);
    if (smac && sst(skb, 6, 6, smac)) return OR_DROP_WRITE_ERROR;
    if (sst(skb, 0, 6, dmac)) return OR_DROP_WRITE_ERROR;
    return OR_TC_ACT_OK;
}

/* ipv6_store_flowlabel (ipv6.h:245-260) of pass_to_stack: version 6, the packet's
 * traffic class, flow label |= SECLABEL_NB (pkg/endpoint/bpf.go:174: htonl(identity)) */
static void ipv6_store_flowlabel(or_skb *skb, uint32_t seclabel)
{
    uint32_t w; memcpy(&w, skb->b + ETH_HLEN, 4);
    const uint32_t label = __builtin_bswap32(seclabel);
    w = __builtin_bswap32(0x60000000u) | label | (w & __builtin_bswap32(0x0FF00000u));
    memcpy(skb->b + ETH_HLEN, &w, 4);
}

/* ipv6_policy (bpf_lxc.c:721-849) + tail_ipv6_policy (:851-862) */
static int ipv6_policy(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t ifindex, uint32_t src_label,
                       int skip_proxy, uint32_t now, pkt_state *ps, int32_t *reason)
{
    int ret, verdict;
    uint32_t len = skb->len;
    if (len < ETH_HLEN + 40) { ret = OR_DROP_INVALID; goto drop; }
    or_ipv6_ct_tuple t; memset(&t, 0, sizeof(t));
    or_ct_state st, st_new; memset(&st, 0, sizeof(st)); memset(&st_new, 0, sizeof(st_new));
    t.nexthdr = skb->b[20];
    memcpy(t.daddr, skb->b + 38, 16); memcpy(t.saddr, skb->b + 22, 16);
    ret = ipv6_hdrlen(skb, ETH_HLEN, &t.nexthdr);
    if (ret < 0) goto drop;
    int l4_off = ETH_HLEN + ret;
    /* derive reverse NAT index and zero it (:750-766): low 16 bits of daddr word 3 */
    uint32_t w3; memcpy(&w3, skb->b + 38 + 12, 4);
    st_new.rev_nat_index = (uint16_t)(w3 & 0xFFFF);
    if (st_new.rev_nat_index) {
        w3 &= ~0xFFFFu;
        int r = sst(skb, ETH_HLEN + 24 + 12, 4, &w3);
        if (r) { ret = r == OR_E_TRUNC ? r : OR_DROP_WRITE_ERROR; goto drop; }
        int coff; uint32_t cfl;                     /* csum_diff(&rev_nat_index, 4, &zero, 4, 0) */
        l4_csum_off(t.nexthdr, &coff, &cfl);
        if (coff && (r = l4_csum_replace(skb, l4_off + coff, 0, csum_diff4(st_new.rev_nat_index, 0, 0),
                                         cfl | OR_F_PSEUDO_HDR))) {
            ret = csum_err(r, OR_DROP_CSUM_L4);
            goto drop;
        }
    }
    int mon = 0;
    ret = ct_lookup6(ep->ct6, &t, skb, l4_off, OR_CT_INGRESS, &st, now, dp->flags, &ps->nl, &ps->nu, &mon);
    if (ret < 0) goto drop;
    ps->ct = (uint8_t)ret;
    if (st.rev_nat_index) {
        int r2 = lb6_rev_nat(dp, skb, l4_off, st.rev_nat_index, &t, &ps->nl);
        if (r2 == OR_E_TRUNC || IS_ERR(r2)) { ret = r2; goto drop; }
    }
    verdict = policy_can_access_ingress(ep->policy, dp->flags, len, src_label, t.dport, t.nexthdr, &ps->nl, &ps->nu);
    if (ret != OR_CT_REPLY && ret != OR_CT_RELATED && verdict < 0) {
        if (ret == OR_CT_ESTABLISHED) {
            if (or_map_delete(ep->ct6, &t) == 0) ps->nu += or_ctu;
        }
        ret = OR_DROP_POLICY;
        goto drop;
    }
    if (skip_proxy) verdict = 0;
    if (ret == OR_CT_NEW) {
        st_new.orig_dport = t.dport;
        st_new.src_sec_id = src_label;
        int r = ct_create6(ep->ct6, &t, len, OR_CT_INGRESS, &st_new, now);
        ps->nu += 2 * or_ctu;
        if (IS_ERR(r)) { ret = r; goto drop; }
    }
    if (verdict > 0 && (ret == OR_CT_NEW || ret == OR_CT_ESTABLISHED)) {
        notify_trace(dp, TRACE_TO_PROXY, len, ep->lxc_id, ep->seclabel, 0, 0, HOST_IFINDEX, (uint8_t)ret, mon);
        ps->proxy = (uint16_t)verdict;                /* ipv6_redirect_to_host_port */
        ifindex = HOST_IFINDEX;
    } else {
        update_metrics(dp, len, 1, 0);                /* TRACE_TO_LXC */
        notify_trace(dp, TRACE_TO_LXC, len, ep->lxc_id, src_label, ep->seclabel, ep->lxc_id, ifindex,
                     (uint8_t)ret, mon);
    }
    return ifindex ? OR_TC_ACT_REDIRECT : OR_TC_ACT_OK;
drop:
    if (ret == OR_E_TRUNC) return ret;
    update_metrics(dp, len, 1, (uint8_t)(-ret));      /* tail_ipv6_policy: send_drop_notify */
    notify_drop(dp, ret, len, ep->lxc_id, src_label, ep->seclabel, ep->lxc_id, ifindex);
    if (reason) *reason = ret;
    return OR_TC_ACT_SHOT;
}

/* handle_ipv6 of bpf_netdev (bpf/bpf_netdev.c:172-276), HANDLE_NS and FROM_HOST as in
 * netdev_config.h, ENCAP_IFINDEX paths (overlay) disabled, reverse_proxy6 (:66-125)
 * with an empty cilium_proxy6 map (L7 out of scope).  As handle_ipv4: *final = 1 once
 * the endpoint's policy program ran (its verdict is final). */
static int handle_ipv6(or_dp *dp, or_skb *skb, uint32_t src_identity, int skip_proxy, uint32_t now,
                       uint32_t *out_identity, pkt_state *ps, int *final, int32_t *reason)
{
    *final = 0;
    *out_identity = src_identity;
    if (skb->len < ETH_HLEN + 40) return OR_DROP_INVALID;          /* revalidate_data */
    uint8_t nexthdr = skb->b[20];
    int hdrlen = ipv6_hdrlen(skb, ETH_HLEN, &nexthdr);
    if (hdrlen < 0) return hdrlen;
    int l4_off = ETH_HLEN + hdrlen;
    if (nexthdr == 58) {                                           /* HANDLE_NS: icmp6_handle (icmp6.h:390-412) */
        uint8_t type;                                              /* icmp6_load_type: load_byte(nh_off + 40) */
        int r = sld(skb, ETH_HLEN + 40, 1, &type);
        if (r == OR_E_TRUNC) return r;
        if (r) return OR_E_LDABS;
        if (type == 135) return OR_E_PUNT;                         /* icmp6_handle_ns: tail call */
        if (type == 128 && !memcmp(skb->b + 38, dp->router_ip6, 16)) return OR_E_PUNT;   /* icmp6_send_echo_reply */
    }
    if (src_identity < HEALTH_ID) {                                /* identity_is_reserved (policy.h:46-49) */
        or_remote_endpoint_info *info = ipcache_lookup6(dp, skb->b + 22, 128, &ps->nl);
        if (info && info->sec_label && info->sec_label != CLUSTER_ID) src_identity = info->sec_label;
    }
    *out_identity = src_identity;
    uint32_t flowlabel = WORLD_ID;                                 /* derive_sec_ctx (:50-64) */
    if (!memcmp(skb->b + 22, dp->router_ip6, 8)) {                 /* ipv6_match_prefix_64 (ipv6.h:166-175) */
        uint32_t w; memcpy(&w, skb->b + ETH_HLEN, 4);
        flowlabel = bswap32(w) & 0x000FFFFFu;                      /* bpf_ntohl(*tmp & IPV6_FLOWLABEL_MASK) */
    }
    if (dp->flags & OR_F_FROM_HOST) {
        flowlabel = src_identity;
        const uint8_t nh0 = skb->b[20];                            /* reverse_proxy6 gets ip6->nexthdr */
        if (nh0 == 6 || nh0 == 17) {                               /* port load at l4_off (:79-89) */
            uint8_t p[4];
            int r = sld(skb, l4_off, 4, p);
            if (r == OR_E_TRUNC) return r;
            if (r) return OR_DROP_CT_INVALID_HDR;
        }
        sst(skb, 0, 6, dp->net_mac);                               /* rewrite_dmac_to_host (:156-169) */
    }
    or_endpoint_info *ep = lookup_ip6_endpoint(dp, skb->b + 38, &ps->nl);
    if (ep) {
        if (ep->flags & 1) return OR_TC_ACT_OK;                    /* ENDPOINT_F_HOST */
        /* ipv6_local_delivery (l3.h:71-101): ipv6_l3 -> hop limit, MACs */
        int rl3 = ipv6_l3(skb, ep->node_mac, ep->mac);
        if (rl3 != OR_TC_ACT_OK) return rl3;
        or_endpoint_prog *prog = find_ep(dp, ep->lxc_id);
        if (!prog) return OR_DROP_MISSED_TAIL_CALL;               /* tail_call(cilium_policy, lxc_id) missed */
        *final = 1;
        return handle_policy(dp, prog, skb, ep->ifindex, flowlabel, skip_proxy, now, ps, reason);
    }
    return OR_TC_ACT_OK;
}

/* handle_ipv6 (bpf_lxc.c:360-387) + ipv6_l3_from_lxc (:82-352), direct routing */
static int handle_ipv6_from_lxc(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t hash, uint32_t now,
                                uint32_t *dst_id, pkt_state *ps, int *final, int32_t *reason)
{
    or_ipv6_ct_tuple t; memset(&t, 0, sizeof(t));
    or_ct_state st_new, st; memset(&st_new, 0, sizeof(st_new)); memset(&st, 0, sizeof(st));
    or_lb6_key key; memset(&key, 0, sizeof(key));
    uint32_t len = skb->len;
    uint8_t *f = skb->b;
    int ret, verdict;
    *final = 0;
    if (!ep->ct6) return OR_DROP_MISSED_TAIL_CALL;                  /* endpoint without an IPv6 program */
    if (len < ETH_HLEN + 40) return OR_DROP_INVALID;
    if (f[20] == 58) {                                              /* icmp6_handle (icmp6.h:390-412) */
        if (len < ETH_HLEN + 40 + 8) return OR_DROP_INVALID;
        uint8_t type = f[54];
        if (type == 135) return OR_E_PUNT;                          /* icmp6_handle_ns tail call */
        if (type == 128 && !memcmp(f + 38, dp->router_ip6, 16)) return OR_E_PUNT;   /* echo reply */
    }
    t.nexthdr = f[20];
    if (memcmp(f + 6, ep->mac, 6)) return OR_DROP_INVALID_SMAC;
    if (memcmp(f + 0, ep->node_mac, 6)) return OR_DROP_INVALID_DMAC;
    if (memcmp(f + 22, ep->ipv6, 16)) return OR_DROP_INVALID_SIP;  /* is_valid_lxc_src_ip (:41-49) */
    memcpy(t.daddr, f + 38, 16); memcpy(t.saddr, f + 22, 16);
    ret = ipv6_hdrlen(skb, ETH_HLEN, &t.nexthdr);
    if (ret < 0) return ret;
    int l4_off = ETH_HLEN + ret;
    memcpy(key.address, t.daddr, 16);                               /* lb6_extract_key (lb.h:334-349) */
    ret = extract_l4_port(skb, t.nexthdr, l4_off, &key.dport);
    if (ret == OR_E_TRUNC) return ret;
    if (IS_ERR(ret)) {
        if (ret != OR_DROP_UNKNOWN_L4) return ret;
    } else {
        st_new.orig_dport = key.dport;
        or_lb6_service *svc = lb6_lookup_service(dp->lb6_services, &key, &ps->nl);
        if (svc) {
            ret = lb6_local(dp, ep->ct6, skb, l4_off, &key, &t, svc, &st_new, hash, now, ps);
            if (ret == OR_E_TRUNC || IS_ERR(ret)) return ret;
        }
    }
    uint8_t orig_dip[16]; memcpy(orig_dip, t.daddr, 16);
    int mon = 0;
    ret = ct_lookup6(ep->ct6, &t, skb, l4_off, OR_CT_EGRESS, &st, now, dp->flags, &ps->nl, &ps->nu, &mon);
    if (ret < 0) return ret;
    ps->ct = (uint8_t)ret;
    uint32_t dst = WORLD_ID;
    or_remote_endpoint_info *info = ipcache_lookup6(dp, orig_dip, 128, &ps->nl);
    if (info && info->sec_label) dst = info->sec_label;
    else if (!memcmp(skb->b + 38, dp->router_ip6, 8)) dst = CLUSTER_ID;   /* ipv6_match_prefix_64 */
    *dst_id = dst;
    verdict = policy_can_egress(ep->policy, dp->flags, len, dst, t.dport, t.nexthdr, &ps->nl, &ps->nu);
    if (ret != OR_CT_REPLY && ret != OR_CT_RELATED && verdict < 0) {
        if (ret == OR_CT_ESTABLISHED) {
            if (or_map_delete(ep->ct6, &t) == 0) ps->nu += or_ctu;
        }
        return verdict;
    }
    switch (ret) {
    case OR_CT_NEW: {
        st_new.src_sec_id = ep->seclabel;
        int r = ct_create6(ep->ct6, &t, len, OR_CT_EGRESS, &st_new, now);
        ps->nu += 2 * or_ctu;
        if (IS_ERR(r)) return r;
        break;
    }
    case OR_CT_ESTABLISHED:
        break;
    case OR_CT_RELATED: case OR_CT_REPLY:
        if (st.rev_nat_index) {
            int r = lb6_rev_nat(dp, skb, l4_off, st.rev_nat_index, &t, &ps->nl);
            if (r == OR_E_TRUNC || IS_ERR(r)) return r;
        }
        break;
    default:
        return OR_DROP_POLICY;
    }
    if (verdict > 0) {
        notify_trace(dp, TRACE_TO_PROXY, len, ep->lxc_id, ep->seclabel, 0, 0, HOST_IFINDEX, ps->ct, mon);
        ps->proxy = (uint16_t)verdict;                              /* ipv6_redirect_to_host_port */
        int r = ipv6_l3(skb, ep->node_mac, dp->host_mac);
        if (r != OR_TC_ACT_OK) return r;
        return OR_TC_ACT_REDIRECT;
    }
    or_endpoint_info *dep = lookup_ip6_endpoint(dp, skb->b + 38, &ps->nl);
    if (dep) {
        /* to_host: ipv6_l3(NODE_MAC, HOST_IFINDEX_MAC); local: ipv6_local_delivery (l3.h:
         * 71-101) ipv6_l3(endpoint_info.node_mac, endpoint_info.mac) */
        int r = (dep->flags & 1) ? ipv6_l3(skb, ep->node_mac, dp->host_mac) : ipv6_l3(skb, dep->node_mac, dep->mac);
        if (r != OR_TC_ACT_OK) return r;
        update_metrics(dp, len, 2, 0);
        if (dep->flags & 1) {
            notify_trace(dp, TRACE_TO_HOST, len, ep->lxc_id, ep->seclabel, HOST_ID, 0, HOST_IFINDEX, ps->ct, mon);
            return OR_TC_ACT_REDIRECT;
        }
        or_endpoint_prog *prog = find_ep(dp, dep->lxc_id);
        if (!prog) return OR_DROP_MISSED_TAIL_CALL;
        *final = 1;
        if (dp->split) {                                            /* (or_lxc_egress_split) */
            dp->pend_ep = (int32_t)(prog - dp->ep);
            dp->pend_ifindex = dep->ifindex;
            dp->pend_label = ep->seclabel;
            return OR_E_DEFER;
        }
        uint8_t ct_egress = ps->ct;
        r = handle_policy(dp, prog, skb, dep->ifindex, ep->seclabel, 0, now, ps, reason);
        ps->ct = ct_egress;
        return r;
    }
    int r = ipv6_l3(skb, NULL, ep->node_mac);                       /* pass_to_stack */
    if (r != OR_TC_ACT_OK) return r;
    ipv6_store_flowlabel(skb, ep->seclabel);
    update_metrics(dp, len, 2, 0);
    notify_trace(dp, TRACE_TO_STACK, len, ep->lxc_id, ep->seclabel, dst, 0, 0, ps->ct, mon);
    return OR_TC_ACT_OK;
}

/* handle_ingress (bpf_lxc.c:672-716, "from-container") + tail_handle_ipv{4,6}
 * (:382-392, 651-661): the verdict of one packet from endpoint ep */
static int from_container(or_dp *dp, or_endpoint_prog *ep, or_skb *skb, uint32_t hash, uint32_t now,
                          uint32_t *dst_id, pkt_state *ps, int32_t *reason)
{
    uint16_t proto = 0;
    if (skb->avail >= 14) memcpy(&proto, skb->b + 12, 2);           /* skb->protocol */
    int ret, final = 0;
    notify_trace(dp, TRACE_FROM_LXC, skb->len, ep->lxc_id, ep->seclabel, 0, 0, 0, 0, 1);
    if (dp->flags & OR_F_DROP_ALL) {
        if (proto == 0x0608) return OR_E_PUNT;                      /* ARP responder */
        ret = OR_DROP_POLICY;
    } else if (proto == 0xDD86) {
        ret = handle_ipv6_from_lxc(dp, ep, skb, hash, now, dst_id, ps, &final, reason);
    } else if (proto == 0x0008) {
        if (!ep->ipv4) ret = OR_DROP_MISSED_TAIL_CALL;              /* no CILIUM_CALL_IPV4_FROM_LXC */
        else ret = handle_ipv4_from_lxc(dp, ep, skb, hash, now, dst_id, ps, &final, reason);
    } else if (proto == 0x0608) {
        return OR_E_PUNT;
    } else {
        ret = OR_DROP_UNKNOWN_L3;
    }
    if (final || ret == OR_E_TRUNC || ret == OR_E_PUNT) return ret;
    if (IS_ERR(ret)) {                                              /* send_drop_notify(METRIC_EGRESS) */
        update_metrics(dp, skb->len, 2, (uint8_t)(-ret));
        notify_drop(dp, ret, skb->len, ep->lxc_id, ep->seclabel, 0, 0, 0);
        *reason = ret;
        return OR_TC_ACT_SHOT;
    }
    return ret;
}

static void lxc_egress(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                       const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash, uint32_t n,
                       uint32_t now, or_out *out, int32_t *dl_ep, uint32_t *dl_ifindex, uint32_t *dl_label)
{
    or_skb skb;
    dp->split = dl_ep != NULL;
    for (uint32_t i = 0; i < n; i++) {
        skb_init(&skb, frames + (size_t)i * stride, stride, len[i]);
        pkt_state ps = { OR_CT_NONE, 0, 0, 0 };
        dp->cur_pkt = i;
        dp->pend_ep = -1;
        dp->cur_hash = flow_hash ? flow_hash[i] : 0;   /* get_hash_recalc(skb) */
        uint32_t e = src_ep ? src_ep[i] : ep0, dst = 0;
        int32_t reason = 0, ret;
        if (e >= dp->n_ep) ret = OR_DROP_MISSED_TAIL_CALL;
        else ret = from_container(dp, &dp->ep[e], &skb, flow_hash ? flow_hash[i] : 0, now, &dst, &ps, &reason);
        if (out->ret) out->ret[i] = ret;
        if (out->identity) out->identity[i] = dst;
        if (out->ct) out->ct[i] = ps.ct;
        if (out->proxy) out->proxy[i] = ps.proxy;
        if (out->nl) out->nl[i] = ps.nl;
        if (out->nu) out->nu[i] = ps.nu;
        if (out->reason) out->reason[i] = reason;
        if (out->xdp) out->xdp[i] = 0;
        emit_frame(out, i, frames + (size_t)i * stride, stride, &skb, ret, ps.proxy);
        if (dl_ep) {
            dl_ep[i] = ret == OR_E_DEFER ? dp->pend_ep : -1;
            dl_ifindex[i] = dp->pend_ifindex;
            dl_label[i] = dp->pend_label;
            if (ret == OR_E_DEFER && out->frames_out) memcpy(out->frames_out + (size_t)i * stride, skb.b, skb.avail);
        }
    }
    dp->split = 0;
}

void or_lxc_egress(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                   const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash, uint32_t n,
                   uint32_t now, or_out *out)
{
    lxc_egress(dp, frames, stride, len, src_ep, ep0, flow_hash, n, now, out, NULL, NULL, NULL);
}

void or_lxc_egress_split(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                         const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash, uint32_t n,
                         uint32_t now, or_out *out, int32_t *dl_ep, uint32_t *dl_ifindex, uint32_t *dl_label)
{
    lxc_egress(dp, frames, stride, len, src_ep, ep0, flow_hash, n, now, out, dl_ep, dl_ifindex, dl_label);
}

void or_lxc_deliver(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len, const int32_t *dl_ep,
                    const uint32_t *dl_ifindex, const uint32_t *dl_label, const uint32_t *pkt, uint32_t n,
                    uint32_t now, or_out *out)
{
    or_skb skb;
    for (uint32_t j = 0; j < n; j++) {
        skb_init(&skb, frames + (size_t)j * stride, stride, len[j]);
        pkt_state ps = { OR_CT_NONE, 0, out->nl ? out->nl[j] : 0, out->nu ? out->nu[j] : 0 };
        dp->cur_pkt = pkt ? pkt[j] : j;
        int32_t reason = 0;
        const int ret = handle_policy(dp, &dp->ep[dl_ep[j]], &skb, dl_ifindex[j], dl_label[j], 0, now, &ps, &reason);
        if (out->ret) out->ret[j] = ret;
        if (out->proxy) out->proxy[j] = ps.proxy;
        if (out->nl) out->nl[j] = ps.nl;
        if (out->nu) out->nu[j] = ps.nu;
        if (out->reason) out->reason[j] = reason;
        emit_frame(out, j, frames + (size_t)j * stride, stride, &skb, ret, ps.proxy);
    }
}

/* ctmap.GC with GCFilterByTime / Flush (pkg/maps/ctmap/ctmap.go:325-432): every
 * entry whose ct_entry.lifetime (u32 @32, host order) is below `time` is deleted
 * (doFiltering, :400-408).  Flush is time = MaxTime.  Returns the number deleted. */
uint32_t or_ct_gc(or_map *m, uint32_t time)
{
    if (!m || m->vs < 36) return 0;
    const uint32_t n = or_map_count(m);
    if (!n) return 0;
    uint8_t *keys = malloc((size_t)n * m->ks), *vals = malloc((size_t)n * m->vs);
    const uint32_t got = or_map_dump(m, keys, vals, n);
    uint32_t deleted = 0;
    for (uint32_t i = 0; i < got; ++i) {
        uint32_t lifetime;
        memcpy(&lifetime, vals + (size_t)i * m->vs + 32, 4);
        if (lifetime < time && or_map_delete(m, keys + (size_t)i * m->ks) == 0) ++deleted;
    }
    free(keys);
    free(vals);
    return deleted;
}

/* known-answer access to the checksum restatement (tests/test_oracle_golden.py):
 * op 0 l3_csum_replace, 1 l4_csum_replace on frame[0..len), 2 csum_diff4 -> *diff,
 * 3 csum_diff16(frame[0..16), frame[16..32), seed = flags) -> *diff */
int or_csum_apply(uint8_t *frame, uint32_t len, uint32_t op, uint32_t off, uint32_t from, uint32_t to,
                  uint32_t flags, uint64_t *diff)
{
    if (op == 2) { *diff = csum_diff4(from, to, flags); return 0; }
    if (op == 3) { *diff = csum_diff16(frame, frame + 16, flags); return 0; }   /* frame = from16 | to16 */
    or_skb s;
    skb_init(&s, frame, len, len);
    int r = op == 0 ? l3_csum_replace(&s, (int)off, from, to, (int)(flags & 0xF))
                    : l4_csum_replace(&s, (int)off, from, to, flags);
    memcpy(frame, s.b, s.avail);
    return r;
}
