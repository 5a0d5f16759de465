// cv_agent.cpp — the reference agent's prefilter and policy-map sync state machines
// (include/cilium_agent.h), restated in C++ over the engine's C-ABI map calls.
//
// PreFilter:      pkg/policy/prefilter.go:57-298 over pkg/maps/cidrmap/cidrmap.go:57-140
// syncPolicyMap:  pkg/endpoint/endpoint.go:2524-2604 over pkg/maps/policymap/policymap.go:146-240
#include <errno.h>
#include <stdio.h>
#include <string.h>

#include <array>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cilium_agent.h"

namespace {

constexpr uint32_t MAX_LKEYS = 1024 * 64;          // prefilter.go:43-44
constexpr uint32_t MAX_HKEYS = 1024 * 1024 * 20;
constexpr uint32_t BPF_F_NO_PREALLOC = 1;
const char *const MAP_NAMES[4] = {"cilium_cidr_v4_dyn", "cilium_cidr_v4_fix", "cilium_cidr_v6_dyn",
                                  "cilium_cidr_v6_fix"};   // cidrmap.MapName + suffix (prefilter.go:214-238)
const int ROLES[4] = {CV_ROLE_CIDR4_DYN, CV_ROLE_CIDR4_FIX, CV_ROLE_CIDR6_DYN, CV_ROLE_CIDR6_FIX};

void set_err(char *err, uint32_t len, const std::string &m)
{
    if (err && len) snprintf(err, len, "%s", m.c_str());
}

// net.IPNet.String(): "10.0.0.0/8", "fd00::a:1/128" (Go's IPv6 form: longest zero
// run of >= 2 groups as "::", lowercase hex)
std::string cidr_str(const cv_cidr &c)
{
    char b[64];
    if (c.family == 4) {
        snprintf(b, sizeof b, "%u.%u.%u.%u/%u", c.addr[0], c.addr[1], c.addr[2], c.addr[3], c.prefixlen);
        return b;
    }
    uint16_t g[8];
    for (int i = 0; i < 8; ++i) g[i] = (uint16_t)(c.addr[2 * i] << 8 | c.addr[2 * i + 1]);
    int bs = -1, bl = 0;
    for (int i = 0; i < 8;) {
        if (g[i]) { ++i; continue; }
        int j = i;
        while (j < 8 && !g[j]) ++j;
        if (j - i > bl) { bs = i; bl = j - i; }
        i = j;
    }
    if (bl < 2) bs = -1;
    std::string s;
    for (int i = 0; i < 8; ++i) {
        if (i == bs) { s += "::"; i += bl - 1; continue; }
        if (!s.empty() && s.back() != ':') s += ":";
        snprintf(b, sizeof b, "%x", g[i]);
        s += b;
    }
    snprintf(b, sizeof b, "/%u", c.prefixlen);
    return s + b;
}

}  // namespace

// ============================================================== prefilter
struct cv_prefilter {
    cv_ctx *ctx;
    int maps[4];               // handle per preFilterMapType, -1 = nil
    bool bound[4];             // bound to its CV_ROLE_* here
    uint32_t config;
    int64_t revision;
    std::mutex mu;             // PreFilter.mutex
};

namespace {

int addr_size(int which) { return which < CV_PF_V6_DYN ? 4 : 16; }
bool is_dyn(int which) { return which == CV_PF_V4_DYN || which == CV_PF_V6_DYN; }

// selectMap (prefilter.go:108-122): bits = 32 or 128 from the family
int select_map(const cv_cidr &c)
{
    const int bits = c.family == 4 ? 32 : c.family == 6 ? 128 : 0;
    if (bits == 32) return c.prefixlen == 32 ? CV_PF_V4_FIX : CV_PF_V4_DYN;
    if (bits == 128) return c.prefixlen == 128 ? CV_PF_V6_FIX : CV_PF_V6_DYN;
    return 4;   // mapCount
}

// cidrKeyInit (cidrmap.go:57-64): {u32 prefixlen, the address's AddrSize bytes}
std::vector<uint8_t> cidr_key(int which, const cv_cidr &c)
{
    const int as = addr_size(which);
    std::vector<uint8_t> k(4 + as);
    const uint32_t pl = c.prefixlen;
    memcpy(k.data(), &pl, 4);
    memcpy(k.data() + 4, c.addr, as);
    return k;
}

// checkPrefixlen (cidrmap.go:75-85): a fix map's Prefixlen is the full length, a dyn
// map's is 0 (OpenMapElems: prefix = 0 when dynamic), so only fix maps check
int check_prefixlen(int which, const cv_cidr &c, const char *op, std::string &msg)
{
    if (is_dyn(which)) return 0;
    const uint32_t want = 8u * (uint32_t)addr_size(which);
    if (c.prefixlen == want) return 0;
    char b[160];
    snprintf(b, sizeof b, "Unable to %s element with dynamic prefix length cm.Prefixlen=%u key.Prefixlen=%u", op,
             want, (unsigned)c.prefixlen);
    msg = b;
    return -EINVAL;
}

int insert_cidr(cv_prefilter *p, int which, const cv_cidr &c, std::string &msg)   // cidrmap.go:87-96
{
    int r = check_prefixlen(which, c, "update", msg);
    if (r) return r;
    const std::vector<uint8_t> k = cidr_key(which, c);
    const uint8_t v = 0;
    r = cv_map_update(p->ctx, p->maps[which], k.data(), &v, CV_ANY);
    if (r) msg = strerror(-r);
    return r;
}

int delete_cidr(cv_prefilter *p, int which, const cv_cidr &c, std::string &msg)   // cidrmap.go:98-106
{
    int r = check_prefixlen(which, c, "delete", msg);
    if (r) return r;
    const std::vector<uint8_t> k = cidr_key(which, c);
    r = cv_map_delete(p->ctx, p->maps[which], k.data());
    if (r) msg = strerror(-r);
    return r;
}

// CIDRExists (cidrmap.go:108-113): a map lookup -- on the LPM trie a longest-prefix
// match, so a covering shorter prefix also "exists"
bool cidr_exists(cv_prefilter *p, int which, const cv_cidr &c)
{
    const std::vector<uint8_t> k = cidr_key(which, c);
    uint8_t v;
    return cv_map_lookup(p->ctx, p->maps[which], k.data(), &v) == 0;
}

std::string revision_msg(int64_t have, int64_t want)
{
    char b[96];
    snprintf(b, sizeof b, "Latest revision is %lld not %lld", (long long)have, (long long)want);
    return b;
}

}  // namespace

extern "C" {

int cv_prefilter_new(cv_ctx *ctx, uint32_t config, cv_prefilter **out)
{
    if (!ctx || !out) return -EINVAL;
    auto *p = new cv_prefilter;
    p->ctx = ctx;
    p->config = config;
    p->revision = 1;
    const bool dyn4 = config & CV_PF_DYN4, fix4 = config & CV_PF_FIX4, dyn6 = config & CV_PF_DYN6,
               fix6 = config & CV_PF_FIX6;
    // initOneMap's skip flags; the v6 fix map follows fix4 (prefilter.go:237)
    const bool make[4] = {dyn4, fix4, dyn6, fix4};
    for (int w = 0; w < 4; ++w) p->maps[w] = -1, p->bound[w] = false;
    for (int w = 0; w < 4; ++w) {
        if (!make[w]) continue;
        const uint32_t ks = 4 + (uint32_t)addr_size(w);
        const int r = cv_map_create(ctx, is_dyn(w) ? CV_MAP_LPM_TRIE : CV_MAP_HASH, ks, 1,
                                    is_dyn(w) ? MAX_LKEYS : MAX_HKEYS, BPF_F_NO_PREALLOC, &p->maps[w]);
        if (r) {
            cv_prefilter_free(p);
            return r;
        }
    }
    // the maps the XDP program built from WriteConfig reads: CIDR4_FILTER (fix4) and,
    // under it, CIDR4_LPM_PREFILTER (dyn4); the same for v6 with the fix6 flag
    const bool bind[4] = {fix4 && dyn4, fix4, fix6 && dyn6, fix6};
    for (int w = 0; w < 4; ++w) {
        if (!bind[w] || p->maps[w] < 0) continue;
        const int r = cv_bind(ctx, ROLES[w], p->maps[w]);
        if (r) {
            cv_prefilter_free(p);
            return r;
        }
        p->bound[w] = true;
    }
    *out = p;
    return 0;
}

void cv_prefilter_free(cv_prefilter *p)
{
    if (!p) return;
    for (int w = 0; w < 4; ++w) {
        if (p->bound[w]) cv_bind(p->ctx, ROLES[w], -1);
        if (p->maps[w] >= 0) cv_map_close(p->ctx, p->maps[w]);
    }
    delete p;
}

int cv_prefilter_map(cv_prefilter *p, int which)
{
    if (!p || which < 0 || which > 3) return -1;
    return p->maps[which];
}

// Insert (prefilter.go:125-159)
int cv_prefilter_insert(cv_prefilter *p, int64_t revision, const cv_cidr *cidrs, uint32_t n, char *err,
                        uint32_t errlen)
{
    if (!p || (n && !cidrs)) return -EINVAL;
    std::lock_guard<std::mutex> g(p->mu);
    if (revision != 0 && p->revision != revision) {
        set_err(err, errlen, revision_msg(p->revision, revision));
        return -ESTALE;
    }
    std::vector<uint32_t> undo;
    int ret = 0;
    std::string msg;
    for (uint32_t i = 0; i < n; ++i) {
        const int w = select_map(cidrs[i]);
        if (w == 4 || p->maps[w] < 0) {
            msg = "No map enabled for CIDR string " + cidr_str(cidrs[i]);
            ret = -EINVAL;
            break;
        }
        std::string why;
        const int r = insert_cidr(p, w, cidrs[i], why);
        if (r) {
            msg = "Error inserting CIDR string " + cidr_str(cidrs[i]) + ": " + why;
            ret = r;
            break;
        }
        undo.push_back(i);
    }
    if (!ret) {
        p->revision++;
        return 0;
    }
    for (uint32_t i : undo) {
        std::string ignored;
        delete_cidr(p, select_map(cidrs[i]), cidrs[i], ignored);
    }
    set_err(err, errlen, msg);
    return ret;
}

// Delete (prefilter.go:162-203)
int cv_prefilter_delete(cv_prefilter *p, int64_t revision, const cv_cidr *cidrs, uint32_t n, char *err,
                        uint32_t errlen)
{
    if (!p || (n && !cidrs)) return -EINVAL;
    std::lock_guard<std::mutex> g(p->mu);
    if (revision != 0 && p->revision != revision) {
        set_err(err, errlen, revision_msg(p->revision, revision));
        return -ESTALE;
    }
    for (uint32_t i = 0; i < n; ++i) {                    // the obvious cases first, before any change
        const int w = select_map(cidrs[i]);
        if (w == 4 || p->maps[w] < 0) {
            set_err(err, errlen, "No map enabled for CIDR string " + cidr_str(cidrs[i]));
            return -EINVAL;
        }
        if (!cidr_exists(p, w, cidrs[i])) {
            set_err(err, errlen, "No map entry for CIDR string " + cidr_str(cidrs[i]));
            return -ENOENT;
        }
    }
    std::vector<uint32_t> undo;
    int ret = 0;
    std::string msg;
    for (uint32_t i = 0; i < n; ++i) {
        std::string why;
        const int r = delete_cidr(p, select_map(cidrs[i]), cidrs[i], why);
        if (r) {
            msg = "Error deleting CIDR string " + cidr_str(cidrs[i]) + ": " + why;
            ret = r;
            break;
        }
        undo.push_back(i);
    }
    if (!ret) {
        p->revision++;
        return 0;
    }
    for (uint32_t i : undo) {
        std::string ignored;
        insert_cidr(p, select_map(cidrs[i]), cidrs[i], ignored);
    }
    set_err(err, errlen, msg);
    return ret;
}

// Dump (prefilter.go:91-106) with cidrmap.CIDRDump / CIDRNext (cidrmap.go:115-140):
// each map walked from the zero key
int cv_prefilter_dump(cv_prefilter *p, cv_cidr *out, uint32_t cap, int64_t *revision)
{
    if (!p) return -EINVAL;
    std::lock_guard<std::mutex> g(p->mu);
    uint32_t n = 0;
    for (int w = 0; w < 4; ++w) {
        if (p->maps[w] < 0) continue;
        const int as = addr_size(w);
        std::vector<uint8_t> key(4 + as, 0), next(4 + as);
        while (cv_map_get_next_key(p->ctx, p->maps[w], key.data(), next.data()) == 0) {
            if (out && n < cap) {                             // keyCidrInit (cidrmap.go:66-73)
                cv_cidr c;
                memset(&c, 0, sizeof c);
                c.family = as == 4 ? 4 : 6;
                uint32_t pl;
                memcpy(&pl, next.data(), 4);
                c.prefixlen = (uint8_t)pl;
                memcpy(c.addr, next.data() + 4, as);
                out[n] = c;
            }
            ++n;
            key = next;
        }
    }
    if (revision) *revision = p->revision;
    return (int)n;
}

// WriteConfig (prefilter.go:65-89); a nil map's String() is "" and path.Base("") "."
int cv_prefilter_write_config(cv_prefilter *p, char *buf, uint32_t len)
{
    if (!p) return -EINVAL;
    std::lock_guard<std::mutex> g(p->mu);
    auto name = [&](int w) { return std::string(p->maps[w] >= 0 ? MAP_NAMES[w] : "."); };
    char b[128];
    std::string s;
    snprintf(b, sizeof b, "#define CIDR4_HMAP_ELEMS %u\n", MAX_HKEYS);
    s += b;
    snprintf(b, sizeof b, "#define CIDR4_LMAP_ELEMS %u\n", MAX_LKEYS);
    s += b;
    s += "#define CIDR4_HMAP_NAME " + name(CV_PF_V4_FIX) + "\n";
    s += "#define CIDR4_LMAP_NAME " + name(CV_PF_V4_DYN) + "\n";
    s += "#define CIDR6_HMAP_NAME " + name(CV_PF_V6_FIX) + "\n";
    s += "#define CIDR6_LMAP_NAME " + name(CV_PF_V6_DYN) + "\n";
    if (p->config & CV_PF_FIX4) {
        s += "#define CIDR4_FILTER\n";
        if (p->config & CV_PF_DYN4) s += "#define CIDR4_LPM_PREFILTER\n";
    }
    if (p->config & CV_PF_FIX6) {
        s += "#define CIDR6_FILTER\n";
        if (p->config & CV_PF_DYN6) s += "#define CIDR6_LPM_PREFILTER\n";
    }
    if (buf && len) snprintf(buf, len, "%s", s.c_str());
    return (int)s.size();
}

}  // extern "C"

// ============================================================== policy map sync
namespace {

// PolicyMapState keys (host byte order), ordered for the std::map
struct PKey {
    uint32_t id;
    uint16_t dport;
    uint8_t nexthdr, dir;
    bool operator<(const PKey &o) const
    {
        if (id != o.id) return id < o.id;
        if (dport != o.dport) return dport < o.dport;
        if (nexthdr != o.nexthdr) return nexthdr < o.nexthdr;
        return dir < o.dir;
    }
};

uint16_t swap16(uint16_t x) { return (uint16_t)(x << 8 | x >> 8); }

// struct policy_key (bpf/lib/common.h): {u32 sec_label, u16 dport (network), u8
// protocol, u8 egress}; struct policy_entry: {u16 proxy_port (network), 3 x u16 pad,
// u64 packets, u64 bytes}
void key_bytes(const PKey &k, uint8_t out[8])                    // PolicyKey.ToNetwork
{
    const uint16_t np = swap16(k.dport);
    memcpy(out, &k.id, 4);
    memcpy(out + 4, &np, 2);
    out[6] = k.nexthdr;
    out[7] = k.dir;
}

PKey key_host(const uint8_t in[8])                               // PolicyKey.ToHost
{
    PKey k;
    uint16_t np;
    memcpy(&k.id, in, 4);
    memcpy(&np, in + 4, 2);
    k.dport = swap16(np);
    k.nexthdr = in[6];
    k.dir = in[7];
    return k;
}

}  // namespace

struct cv_policy_sync {
    std::map<PKey, uint16_t> desired, realized;                  // PolicyMapStateEntry{ProxyPort}
    std::mutex mu;
};

extern "C" {

int cv_policy_sync_new(cv_policy_sync **out)
{
    if (!out) return -EINVAL;
    *out = new cv_policy_sync;
    return 0;
}

void cv_policy_sync_free(cv_policy_sync *s) { delete s; }

int cv_policy_sync_set_desired(cv_policy_sync *s, const cv_policy_key *keys, const uint16_t *proxy, uint32_t n)
{
    if (!s || (n && (!keys || !proxy))) return -EINVAL;
    std::lock_guard<std::mutex> g(s->mu);
    s->desired.clear();
    for (uint32_t i = 0; i < n; ++i)
        s->desired[PKey{keys[i].identity, keys[i].dport, keys[i].nexthdr, keys[i].direction}] = proxy[i];
    return 0;
}

// Endpoint.syncPolicyMap (pkg/endpoint/endpoint.go:2524-2604)
int cv_policy_sync_run(cv_policy_sync *s, cv_ctx *ctx, int h, uint32_t *deleted, uint32_t *added,
                       uint32_t *failed)
{
    if (!s || !ctx) return -EINVAL;
    std::lock_guard<std::mutex> g(s->mu);
    uint32_t nd = 0, na = 0, nf = 0;
    // policymap.DumpToSlice (policymap.go:208-240): GetNextKey from the zero key, a
    // lookup per key (a failed lookup fails the dump)
    std::vector<std::array<uint8_t, 8>> current;
    {
        uint8_t key[8] = {0}, next[8], val[24];
        while (cv_map_get_next_key(ctx, h, key, next) == 0) {
            const int r = cv_map_lookup(ctx, h, next, val);
            if (r) return r;
            std::array<uint8_t, 8> k;
            memcpy(k.data(), next, 8);
            current.push_back(k);
            memcpy(key, next, 8);
        }
    }
    for (const auto &e : current) {                              // not desired: delete
        const PKey kh = key_host(e.data());
        if (s->desired.count(kh)) continue;
        uint8_t kb[8];
        key_bytes(kh, kb);                                       // DeleteKey: back to network order
        if (cv_map_delete(ctx, h, kb)) {
            ++nf;
        } else {
            s->realized.erase(kh);
            ++nd;
        }
    }
    for (const auto &d : s->desired) {                           // missing or changed: AllowKey
        auto it = s->realized.find(d.first);
        if (it != s->realized.end() && it->second == d.second) continue;
        uint8_t kb[8], vb[24] = {0};
        key_bytes(d.first, kb);
        const uint16_t pp = swap16(d.second);
        memcpy(vb, &pp, 2);
        if (cv_map_update(ctx, h, kb, vb, CV_ANY)) {
            ++nf;
        } else {
            s->realized[d.first] = d.second;
            ++na;
        }
    }
    if (deleted) *deleted = nd;
    if (added) *added = na;
    if (failed) *failed = nf;
    return nf ? -EIO : 0;
}

int cv_policy_sync_realized(cv_policy_sync *s, cv_policy_key *keys, uint16_t *proxy, uint32_t cap)
{
    if (!s) return -EINVAL;
    std::lock_guard<std::mutex> g(s->mu);
    uint32_t n = 0;
    for (const auto &r : s->realized) {
        if (keys && proxy && n < cap) {
            keys[n] = cv_policy_key{r.first.id, r.first.dport, r.first.nexthdr, r.first.dir};
            proxy[n] = r.second;
        }
        ++n;
    }
    return (int)n;
}

}  // extern "C"
