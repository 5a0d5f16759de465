// cv_epnode.cpp — round scheduler of the endpoint-owned node (include/cilium_epnode.h,
// DESIGN.md §7).  Host code: per batch it derives every packet's candidate destinations
// and the peers of its CT operations from the headers and the context's service table,
// lists the operations of the rank's maps in packet order, and per round hands out the
// operations no earlier pending operation blocks.
//
// Blocking is within one CT map: an operation's keys are (its map, a peer address), all
// in its own map, so one in-order scan over a map's pending operations finds the ready
// ones -- a blocked operation stamps its peers, and a later operation meeting a stamped
// peer is blocked in turn; on a map that may fill (`tight`) the first blocked operation
// blocks every later one (conntrack.h:692-693: creates of different peers compete for
// the room).  Peers are 64-bit address hashes folded to PEER_SLOTS stamps: two peers
// folding together only add an ordering constraint, never drop one.
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/cilium_epnode.h"
#include "cv_node.hpp"

namespace {

constexpr uint32_t PEER_SLOTS = 1u << 22;
// the most entries one operation creates in its map: a source program its service entry,
// the connection's tuple, its ICMP-RELATED twin and the NAT tuple (lb{4,6}_local,
// ct_create{4,6}: lb.h:700-775, conntrack.h:663-744) -- bounded by 7 as cv_lxc_egress
// plans launches; a delivery the tuple and its twin (ipv4_policy / ipv6_policy)
constexpr int64_t MAX_CREATES[2] = {7, 2};
enum : uint8_t { OP_PENDING = 0, OP_RESOLVED = 1, OP_DONE = 2 };

struct Addr {
    uint64_t a, b;
    uint32_t fam;
    bool operator==(const Addr &o) const { return a == o.a && b == o.b && fam == o.fam; }
};

inline uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct AddrHash {
    size_t operator()(const Addr &x) const { return (size_t)mix(mix(x.a ^ x.fam) + x.b); }
};

Addr addr4(const uint8_t *p)
{
    uint32_t w;
    memcpy(&w, p, 4);
    return Addr{0, w, 4};
}

Addr addr6(const uint8_t *p)
{
    Addr r{0, 0, 6};
    memcpy(&r.a, p, 8);
    memcpy(&r.b, p + 8, 8);
    return r;
}

inline uint32_t peer_slot(const Addr &x) { return (uint32_t)(AddrHash()(x) & (PEER_SLOTS - 1)); }

}  // namespace

struct cv_epnode {
    cv_ctx *ctx = nullptr;
    uint32_t rank = 0, world = 1, n = 0, n_eps = 0;
    std::vector<uint8_t> v6;
    std::vector<uint32_t> cand_off, cand;          // per packet its candidate destinations (CSR, ascending)
    // operations of this rank in (packet, kind, endpoint) order
    std::vector<uint32_t> op_pkt, op_map, op_poff, op_peer;
    std::vector<uint8_t> op_kind, op_st;
    std::vector<uint32_t> dl_first;                // per packet its first delivery operation here (or ~0)
    std::vector<uint8_t> dl_cnt;
    // per map (endpoint * 2 + family): its operations in order, the first not done
    std::vector<uint32_t> map_off, map_ops, map_head;
    std::vector<int> map_handle;
    std::vector<int64_t> map_need;                 // creates its pending operations may still make
    std::vector<uint64_t> map_live, map_cap;
    std::vector<uint8_t> map_tight;
    std::vector<uint32_t> active;                  // maps with operations
    std::vector<uint32_t> stamp;
    uint32_t cur = 0;
    uint64_t pending = 0, rounds = 0, n_src = 0, n_dl = 0, tight0 = 0, sent = 0;
    cv_epnode_counts_fn counts = nullptr;          // (the caller's live counts, else the context's maps)
    void *counts_arg = nullptr;

    uint32_t next_stamp()
    {
        if (++cur == 0) {                          // (wrapped: forget every stamp)
            std::fill(stamp.begin(), stamp.end(), 0u);
            cur = 1;
        }
        return cur;
    }
    void finish(uint32_t o)
    {
        op_st[o] = OP_DONE;
        map_need[op_map[o]] -= MAX_CREATES[op_kind[o]];
        --pending;
    }
    bool owned(uint32_t ep) const { return ep % world == rank; }
    int refresh_tight(bool all);
    template <class Ready>
    void scan(Ready ready, std::vector<uint32_t> &out);
};

// live + the creates the pending operations may make > max_entries: the map may fill
int cv_epnode::refresh_tight(bool all)
{
    std::vector<int> hs;
    std::vector<uint32_t> ms;
    for (uint32_t m : active)
        if (map_handle[m] >= 0 && (all || map_tight[m])) {
            hs.push_back(map_handle[m]);
            ms.push_back(m);
        }
    if (hs.empty()) return 0;
    std::vector<uint64_t> live(hs.size()), cap(hs.size());
    const int r = counts ? counts(counts_arg, hs.data(), (uint32_t)hs.size(), live.data(), cap.data())
                         : cv::ct_counts(ctx, hs, live, cap);
    if (r) return r;
    for (size_t k = 0; k < ms.size(); ++k) {
        map_live[ms[k]] = live[k];
        map_cap[ms[k]] = cap[k];
        map_tight[ms[k]] = (int64_t)live[k] + std::max<int64_t>(map_need[ms[k]], 0) > (int64_t)cap[k];
    }
    return 0;
}

// one in-order pass over every active map's pending operations; ready(o) says whether
// operation o may run now if nothing earlier blocks it
template <class Ready>
void cv_epnode::scan(Ready ready, std::vector<uint32_t> &out)
{
    for (uint32_t m : active) {
        uint32_t &h = map_head[m];
        const uint32_t end = map_off[m + 1];
        while (h < end && op_st[map_ops[h]] == OP_DONE) ++h;
        if (h == end) continue;
        const uint32_t st = next_stamp();
        for (uint32_t k = h; k < end; ++k) {
            const uint32_t o = map_ops[k];
            if (op_st[o] == OP_DONE) continue;
            bool free = ready(o);
            for (uint32_t q = op_poff[o]; free && q < op_poff[o + 1]; ++q) free = stamp[op_peer[q]] != st;
            if (free) {
                out.push_back(o);
                continue;
            }
            if (map_tight[m]) break;                       // (the map keeps packet order across peers)
            for (uint32_t q = op_poff[o]; q < op_poff[o + 1]; ++q) stamp[op_peer[q]] = st;
        }
    }
    std::sort(out.begin(), out.end(), [&](uint32_t x, uint32_t y) { return op_pkt[x] < op_pkt[y]; });
}

extern "C" {

int cv_epnode_open(cv_ctx *ctx, uint32_t rank, uint32_t world, const uint8_t *frames, uint32_t stride, uint32_t n,
                   const uint16_t *src_ep, cv_epnode **out)
{
    if (!ctx || !out || !world || rank >= world || (n && (!frames || !src_ep)) || stride < 54) return -EINVAL;
    cv::NodeView v;
    int r = cv::node_view(ctx, v);
    if (r) return r;
    const uint32_t ne = (uint32_t)v.eps.size();
    if (ne > 0xFFFF) return -E2BIG;
    {                                                      // every endpoint's CT maps its own
        std::vector<int> hs;
        for (auto &e : v.eps)
            for (int h : {e.ct4, e.ct6})
                if (h >= 0) hs.push_back(h);
        std::sort(hs.begin(), hs.end());
        if (std::adjacent_find(hs.begin(), hs.end()) != hs.end()) return -EINVAL;
    }
    // address -> endpoints; VIP -> backends; backend -> VIPs
    std::unordered_map<Addr, std::vector<uint32_t>, AddrHash> where;
    std::unordered_map<Addr, std::vector<Addr>, AddrHash> backends, vips;
    for (uint32_t e = 0; e < ne; ++e) {
        if (v.eps[e].ipv4) where[Addr{0, v.eps[e].ipv4, 4}].push_back(e);
        static const uint8_t zero[16] = {};
        if (memcmp(v.eps[e].ipv6, zero, 16)) where[addr6(v.eps[e].ipv6)].push_back(e);
    }
    for (auto &s : v.svc) {
        const Addr vip = s.v6 ? addr6(s.vip) : addr4(s.vip), be = s.v6 ? addr6(s.backend) : addr4(s.backend);
        auto &b = backends[vip];
        if (std::find(b.begin(), b.end(), be) == b.end()) b.push_back(be);
        auto &q = vips[be];
        if (std::find(q.begin(), q.end(), vip) == q.end()) q.push_back(vip);
    }
    const Addr lob{0, v.loopback, 4};
    std::unique_ptr<cv_epnode> nd(new cv_epnode());
    nd->ctx = ctx;
    nd->rank = rank;
    nd->world = world;
    nd->n = n;
    nd->n_eps = ne;
    nd->v6.assign(n, 0);
    nd->cand_off.assign(n + 1, 0);
    nd->dl_first.assign(n, ~0u);
    nd->dl_cnt.assign(n, 0);
    nd->op_poff.push_back(0);
    std::vector<uint32_t> c, sp, dp;
    static const std::vector<Addr> none;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *f = frames + (size_t)i * stride;
        const uint32_t s = src_ep[i];
        if (s >= ne) return -EINVAL;
        c.clear();
        sp.clear();
        dp.clear();
        const bool is4 = f[12] == 0x08 && f[13] == 0x00, is6 = f[12] == 0x86 && f[13] == 0xDD;
        nd->v6[i] = is6;
        if (is4 || is6) {
            const Addr sa = is4 ? addr4(f + 26) : addr6(f + 22), da = is4 ? addr4(f + 30) : addr6(f + 38);
            auto bi = backends.find(da);
            const std::vector<Addr> &bes = bi == backends.end() ? none : bi->second;
            auto add_where = [&](const Addr &a) {
                auto w = where.find(a);
                if (w != where.end()) c.insert(c.end(), w->second.begin(), w->second.end());
            };
            add_where(da);
            for (const Addr &b : bes) add_where(b);
            std::sort(c.begin(), c.end());
            c.erase(std::unique(c.begin(), c.end()), c.end());
            // peers: the source program's -- the destination, a VIP's backends, and the
            // loopback address when the client backs the VIP itself; the delivery's -- the
            // source as the source program left it: itself, a VIP it backs (reverse NAT of
            // a reply), or the loopback address
            const bool loop = v.loopback && std::find(bes.begin(), bes.end(), sa) != bes.end();
            sp.push_back(peer_slot(da));
            for (const Addr &b : bes) sp.push_back(peer_slot(b));
            dp.push_back(peer_slot(sa));
            auto vi = vips.find(sa);
            if (vi != vips.end())
                for (const Addr &x : vi->second) dp.push_back(peer_slot(x));
            if (loop) {
                sp.push_back(peer_slot(lob));
                dp.push_back(peer_slot(lob));
            }
        }
        nd->cand.insert(nd->cand.end(), c.begin(), c.end());
        nd->cand_off[i + 1] = (uint32_t)nd->cand.size();
        const uint32_t fam = is6 ? 1 : 0;
        auto add_op = [&](uint32_t kind, uint32_t ep, const std::vector<uint32_t> &ps) {
            nd->op_pkt.push_back(i);
            nd->op_kind.push_back((uint8_t)kind);
            nd->op_map.push_back(ep * 2 + fam);
            nd->op_peer.insert(nd->op_peer.end(), ps.begin(), ps.end());
            nd->op_poff.push_back((uint32_t)nd->op_peer.size());
        };
        if (nd->owned(s)) {
            add_op(0, s, sp);
            nd->n_src++;
        }
        for (uint32_t d : c)
            if (nd->owned(d)) {
                if (nd->dl_first[i] == ~0u) nd->dl_first[i] = (uint32_t)nd->op_pkt.size();
                nd->dl_cnt[i]++;
                add_op(1, d, dp);
                nd->n_dl++;
            }
    }
    const uint32_t nops = (uint32_t)nd->op_pkt.size(), nm = ne * 2;
    nd->op_st.assign(nops, OP_PENDING);
    for (uint32_t o = 0; o < nops; ++o)
        if (nd->op_kind[o] == 0) nd->op_st[o] = OP_RESOLVED;    // (a source program needs no record)
    nd->pending = nops;
    // per map, its operations in order (a stable counting sort by map)
    nd->map_off.assign(nm + 1, 0);
    for (uint32_t o = 0; o < nops; ++o) nd->map_off[nd->op_map[o] + 1]++;
    for (uint32_t m = 0; m < nm; ++m) nd->map_off[m + 1] += nd->map_off[m];
    nd->map_ops.resize(nops);
    {
        std::vector<uint32_t> at(nd->map_off.begin(), nd->map_off.end() - 1);
        for (uint32_t o = 0; o < nops; ++o) nd->map_ops[at[nd->op_map[o]]++] = o;
    }
    nd->map_head.assign(nd->map_off.begin(), nd->map_off.end() - 1);
    nd->map_handle.assign(nm, -1);
    nd->map_need.assign(nm, 0);
    nd->map_live.assign(nm, 0);
    nd->map_cap.assign(nm, 0);
    nd->map_tight.assign(nm, 0);
    for (uint32_t m = 0; m < nm; ++m) {
        if (nd->map_off[m + 1] == nd->map_off[m]) continue;
        nd->active.push_back(m);
        nd->map_handle[m] = (m & 1) ? v.eps[m >> 1].ct6 : v.eps[m >> 1].ct4;
    }
    for (uint32_t o = 0; o < nops; ++o) nd->map_need[nd->op_map[o]] += MAX_CREATES[nd->op_kind[o]];
    nd->stamp.assign(PEER_SLOTS, 0u);
    *out = nd.release();
    return 0;
}

void cv_epnode_close(cv_epnode *nd) { delete nd; }

int cv_epnode_set_counts(cv_epnode *nd, cv_epnode_counts_fn fn, void *arg)
{
    if (!nd || nd->rounds) return -EINVAL;
    nd->counts = fn;
    nd->counts_arg = arg;
    return 0;
}

uint64_t cv_epnode_pending(const cv_epnode *nd) { return nd ? nd->pending : 0; }

int cv_epnode_stats(const cv_epnode *nd, uint64_t stats[6])
{
    if (!nd || !stats) return -EINVAL;
    uint64_t t = 0;
    for (uint32_t m : nd->active) t += nd->map_tight[m];
    stats[0] = nd->rounds;
    stats[1] = nd->n_src;
    stats[2] = nd->n_dl;
    stats[3] = nd->tight0;
    stats[4] = t;
    stats[5] = nd->sent;
    return 0;
}

int cv_epnode_sources(cv_epnode *nd, uint32_t *pkts, uint32_t cap)
{
    if (!nd || (cap && !pkts)) return -EINVAL;
    int r;
    if (!nd->rounds++) {                                   // every map's room, once
        if ((r = nd->refresh_tight(true))) return r;
        for (uint32_t m : nd->active) nd->tight0 += nd->map_tight[m];
    } else {
        bool any = false;
        for (uint32_t m : nd->active) any |= nd->map_tight[m] != 0;
        if (any && (r = nd->refresh_tight(false))) return r;   // (room re-read for the maps that may fill)
    }
    std::vector<uint32_t> out;
    nd->scan([&](uint32_t o) { return nd->op_kind[o] == 0; }, out);
    if (out.size() > cap) return -ENOSPC;
    for (size_t j = 0; j < out.size(); ++j) {
        pkts[j] = nd->op_pkt[out[j]];
        nd->finish(out[j]);
    }
    return (int)out.size();
}

int cv_epnode_sources_done(cv_epnode *nd, const uint32_t *pkts, const int32_t *dst, uint32_t n, uint32_t *row_pkt,
                           uint32_t *row_ep, uint8_t *row_has, uint32_t *row_pos, uint32_t *rank_rows, uint32_t cap)
{
    if (!nd || (n && (!pkts || !dst)) || !rank_rows) return -EINVAL;
    std::vector<uint32_t> cnt(nd->world + 1, 0);
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t i = pkts[j];
        if (i >= nd->n) return -EINVAL;
        const uint32_t *b = nd->cand.data() + nd->cand_off[i], *e = nd->cand.data() + nd->cand_off[i + 1];
        if (dst[j] >= 0 && !std::binary_search(b, e, (uint32_t)dst[j])) return -EPROTO;   // (outside the candidates)
        for (const uint32_t *d = b; d < e; ++d) cnt[*d % nd->world + 1]++;
    }
    for (uint32_t k = 0; k < nd->world; ++k) cnt[k + 1] += cnt[k];
    const uint32_t total = cnt[nd->world];
    if (total > cap) return -ENOSPC;
    if (total && (!row_pkt || !row_ep || !row_has || !row_pos)) return -EINVAL;
    for (uint32_t k = 0; k < nd->world; ++k) {
        rank_rows[k] = cnt[k + 1] - cnt[k];
        if (k != nd->rank) nd->sent += rank_rows[k];
    }
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t i = pkts[j];
        for (uint32_t q = nd->cand_off[i]; q < nd->cand_off[i + 1]; ++q) {
            const uint32_t d = nd->cand[q], at = cnt[d % nd->world]++;
            row_pkt[at] = i;
            row_ep[at] = d;
            row_has[at] = dst[j] == (int32_t)d;
            row_pos[at] = j;
        }
    }
    return (int)total;
}

int cv_epnode_receive(cv_epnode *nd, const uint32_t *row_pkt, const uint32_t *row_ep, const uint8_t *row_has,
                      uint32_t n, int32_t *op)
{
    if (!nd || (n && (!row_pkt || !row_ep || !row_has || !op))) return -EINVAL;
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t i = row_pkt[j];
        if (i >= nd->n || nd->dl_first[i] == ~0u) return -EPROTO;
        uint32_t o = nd->dl_first[i], k = 0;
        while (k < nd->dl_cnt[i] && nd->op_map[o] >> 1 != row_ep[j]) ++k, ++o;
        if (k == nd->dl_cnt[i] || nd->op_st[o] != OP_PENDING) return -EPROTO;
        if (row_has[j]) {
            nd->op_st[o] = OP_RESOLVED;
            op[j] = (int32_t)o;
        } else {
            nd->finish(o);                                 // (delivered elsewhere, or not at all)
            op[j] = -1;
        }
    }
    return 0;
}

int cv_epnode_deliveries(cv_epnode *nd, uint32_t *ops, uint32_t *pkts, uint32_t cap)
{
    if (!nd || (cap && (!ops || !pkts))) return -EINVAL;
    std::vector<uint32_t> out;
    nd->scan([&](uint32_t o) { return nd->op_kind[o] == 1 && nd->op_st[o] == OP_RESOLVED; }, out);
    if (out.size() > cap) return -ENOSPC;
    for (size_t j = 0; j < out.size(); ++j) {
        ops[j] = out[j];
        pkts[j] = nd->op_pkt[out[j]];
        nd->finish(out[j]);
    }
    return (int)out.size();
}

}  // extern "C"
