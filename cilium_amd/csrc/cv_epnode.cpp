// cv_epnode.cpp — round scheduler of the endpoint-owned node (include/cilium_epnode.h,
// DESIGN.md §7).  Host code: per batch it derives every packet's candidate destinations
// and the peers of its CT operations from the headers and the context's service table,
// lists the operations of the rank's maps in packet order, and per round hands out the
// operations no earlier pending operation blocks.
//
// An operation's keys are (its map, a peer address), all in its own map.  It waits for
// the operation before it on each of its keys (a dependency DAG built once per batch,
// predecessors counted per operation, Kahn-style): when an operation runs, its
// successors' counts drop, and a successor of the same kind whose count reaches zero runs
// in the same launch (the launch keeps packet order per address pair).  On a map that
// may fill (`chain`) every operation also waits for the one before it in the map
// (conntrack.h:692-693: creates of different peers compete for the room) until the
// map's room is ample again.  Each key link is used once per batch, so a round costs the
// operations it runs, not the ones still waiting.  Addresses are 64-bit hashes (two
// colliding only add candidates or a dependency, never drop one).
#include <errno.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/cilium_epnode.h"
#include "cv_node.hpp"

namespace {

// the most entries one operation creates in its map: a source program its service entry,
// the connection's tuple, its ICMP-RELATED twin and the NAT tuple (lb{4,6}_local,
// ct_create{4,6}: lb.h:700-775, conntrack.h:663-744) -- bounded by 7 as cv_lxc_egress
// plans launches; a delivery the tuple and its twin (ipv4_policy / ipv6_policy)
constexpr int64_t MAX_CREATES[2] = {7, 2};
enum : uint8_t { OP_PENDING = 0, OP_RESOLVED = 1, OP_NOOP = 2, OP_DONE = 3 };

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

inline uint64_t ahash(const Addr &x) { return mix(mix(x.a ^ ((uint64_t)x.fam << 56)) + x.b) | 1u; }

struct VipPort {
    uint64_t vip;
    uint16_t vport, bport;
    bool operator<(const VipPort &o) const
    {
        return vip != o.vip ? vip < o.vip : vport != o.vport ? vport < o.vport : bport < o.bport;
    }
    bool operator==(const VipPort &o) const { return vip == o.vip && vport == o.vport && bport == o.bport; }
};

// key -> run of values, from (key, value) pairs: an open-addressing index over the
// distinct keys and their values grouped (CSR)
template <class V>
struct Csr {
    std::vector<uint64_t> keys;
    std::vector<uint32_t> lo, hi;
    std::vector<V> val;
    uint64_t mask = 0;
    explicit Csr(std::vector<std::pair<uint64_t, V>> kv)
    {
        std::sort(kv.begin(), kv.end());
        kv.erase(std::unique(kv.begin(), kv.end()), kv.end());
        uint64_t cap = 16;
        while (cap < 2 * kv.size()) cap <<= 1;
        mask = cap - 1;
        keys.assign(cap, 0);
        lo.assign(cap, 0);
        hi.assign(cap, 0);
        val.reserve(kv.size());
        for (size_t k = 0; k < kv.size();) {
            size_t e = k;
            while (e < kv.size() && kv[e].first == kv[k].first) val.push_back(kv[e++].second);
            uint64_t h = kv[k].first & mask;
            while (keys[h]) h = (h + 1) & mask;
            keys[h] = kv[k].first;
            lo[h] = (uint32_t)(val.size() - (e - k));
            hi[h] = (uint32_t)val.size();
            k = e;
        }
    }
    std::pair<uint32_t, uint32_t> find(uint64_t key) const
    {
        for (uint64_t h = key & mask;; h = (h + 1) & mask) {
            if (keys[h] == key) return {lo[h], hi[h]};
            if (!keys[h]) return {0u, 0u};
        }
    }
};

// the node's indexes: address -> endpoints, VIP -> backends, backend -> (VIP, ports), by
// 64-bit address hash (a collision adds candidates or peers, supersets stay exact); built
// once per node view and reused by every batch while the view's key holds
struct NodeIdx {
    cv::NodeKey key;
    cv::NodeView v;
    Csr<uint32_t> where;
    Csr<uint64_t> backends;
    Csr<VipPort> vips;
    uint64_t lob = 0;
    NodeIdx(const cv::NodeKey &k, cv::NodeView &&view, std::vector<std::pair<uint64_t, uint32_t>> ew,
            std::vector<std::pair<uint64_t, uint64_t>> vb, std::vector<std::pair<uint64_t, VipPort>> bv)
        : key(k), v(std::move(view)), where(std::move(ew)), backends(std::move(vb)), vips(std::move(bv)),
          lob(ahash(Addr{0, v.loopback, 4}))
    {
    }
};

std::shared_ptr<const NodeIdx> build_index(cv_ctx *ctx, const cv::NodeKey &key, int &err)
{
    cv::NodeView v;
    if ((err = cv::node_view(ctx, v))) return nullptr;
    const uint32_t ne = (uint32_t)v.eps.size();
    if (ne > 0xFFFF) { err = -E2BIG; return nullptr; }
    {                                                      // every endpoint's CT maps its own
        std::vector<int> hs;
        for (auto &e : v.eps)
            for (int h : {e.ct4, e.ct6})
                if (h >= 0) hs.push_back(h);
        std::sort(hs.begin(), hs.end());
        if (std::adjacent_find(hs.begin(), hs.end()) != hs.end()) { err = -EINVAL; return nullptr; }
    }
    std::vector<std::pair<uint64_t, uint32_t>> ew;                // (address, endpoint)
    std::vector<std::pair<uint64_t, uint64_t>> vb;                // (VIP, backend)
    for (uint32_t e = 0; e < ne; ++e) {
        static const uint8_t zero[16] = {};
        if (v.eps[e].ipv4) ew.push_back({ahash(Addr{0, v.eps[e].ipv4, 4}), e});
        if (memcmp(v.eps[e].ipv6, zero, 16)) ew.push_back({ahash(addr6(v.eps[e].ipv6)), e});
    }
    for (auto &q : v.svc)
        vb.push_back({ahash(q.v6 ? addr6(q.vip) : addr4(q.vip)), ahash(q.v6 ? addr6(q.backend) : addr4(q.backend))});
    // backend -> (VIP, the key's dport, the backend's port): the VIPs a reply may be
    // reverse-NATed to (see the delivery's peers)
    std::vector<std::pair<uint64_t, VipPort>> bv(vb.size());
    for (size_t k = 0; k < vb.size(); ++k) bv[k] = {vb[k].second, VipPort{vb[k].first, v.svc[k].vport, v.svc[k].bport}};
    return std::make_shared<const NodeIdx>(key, std::move(v), std::move(ew), std::move(vb), std::move(bv));
}

// the most recent node's indexes (one context's node per process at a time; another
// context or a changed view rebuilds them)
std::mutex idx_mu;
std::shared_ptr<const NodeIdx> idx_last;

std::shared_ptr<const NodeIdx> node_index(cv_ctx *ctx, int &err)
{
    cv::NodeKey key;
    if ((err = cv::node_key(ctx, key))) return nullptr;
    {
        std::lock_guard<std::mutex> g(idx_mu);
        if (idx_last && idx_last->key == key) return idx_last;
    }
    std::shared_ptr<const NodeIdx> ix = build_index(ctx, key, err);
    if (ix) {
        std::lock_guard<std::mutex> g(idx_mu);
        idx_last = ix;
    }
    return ix;
}

}  // namespace

struct cv_epnode {
    cv_ctx *ctx = nullptr;
    uint32_t rank = 0, world = 1, n = 0, n_eps = 0;
    std::vector<uint8_t> v6;
    std::vector<uint32_t> cand_off, cand;          // per packet its candidate destinations (CSR, ascending)
    // operations of this rank in (packet, kind, endpoint) order; per key reference of an
    // operation, the next operation on that key (or NONE)
    std::vector<uint32_t> op_pkt, op_map, op_poff, op_mpos;
    std::vector<uint32_t> ref_op, ref_next, ref_prev;   // per key reference: its operation, the neighbours on its key
    std::vector<uint8_t> op_kind, op_st;
    std::vector<uint32_t> op_wait;                 // earlier pending operations it waits for
    std::vector<uint32_t> dl_first;                // per packet its first delivery operation here (or NONE)
    std::vector<uint8_t> dl_cnt;
    // per map (endpoint * 2 + family): its operations in order
    std::vector<uint32_t> map_off, map_ops, map_head;
    std::vector<int> map_handle;
    std::vector<int64_t> map_need;                 // creates its pending operations may still make
    std::vector<uint8_t> map_chain;                // may fill: its operations wait for each other in order
    std::vector<uint32_t> active;                  // maps with operations
    std::vector<uint32_t> zero[2];                 // per kind: operations waiting for nothing, not yet run
    uint64_t pending = 0, rounds = 0, n_src = 0, n_dl = 0, chained0 = 0, sent = 0;
    cv_epnode_counts_fn counts = nullptr;          // (the caller's live counts, else the context's maps)
    void *counts_arg = nullptr;

    static constexpr uint32_t NONE = ~0u;
    bool owned(uint32_t ep) const { return ep % world == rank; }
    uint32_t chain_next(uint32_t o) const
    {
        const uint32_t m = op_map[o], k = op_mpos[o] + 1;
        return k < map_off[m + 1] ? map_ops[k] : NONE;
    }
    void release(uint32_t s)
    {
        if (--op_wait[s] == 0) zero[op_kind[s]].push_back(s);
    }
    // operation o has run (or will not run here): its successors wait for one less.  Its
    // successors are in its own map (rel: what becomes free)
    template <class R>
    void finish_core(uint32_t o, R &&rel)
    {
        op_st[o] = OP_DONE;
        map_need[op_map[o]] -= MAX_CREATES[op_kind[o]];
        for (uint32_t q = op_poff[o]; q < op_poff[o + 1]; ++q)
            if (ref_next[q] != NONE) rel(ref_op[ref_next[q]]);
        if (map_chain[op_map[o]]) {
            const uint32_t s = chain_next(o);
            if (s != NONE) rel(s);
        }
    }
    void finish(uint32_t o)
    {
        finish_core(o, [&](uint32_t x) { release(x); });
        --pending;
    }
    // a delivery that runs nowhere here leaves its keys' lists: each successor waits for
    // the predecessor instead, or for nothing more when the predecessor has finished.
    // Everything it touches is in its own map (rel: what becomes free)
    template <class R>
    void splice_core(uint32_t o, R &&rel)
    {
        for (uint32_t q = op_poff[o]; q < op_poff[o + 1]; ++q) {
            const uint32_t pq = ref_prev[q], nq = ref_next[q];
            const bool waits = pq != NONE && op_st[ref_op[pq]] != OP_DONE;   // (o still waited on pq)
            if (pq != NONE) ref_next[pq] = waits ? nq : NONE;
            if (nq != NONE) {
                ref_prev[nq] = waits ? pq : NONE;
                if (!waits) rel(ref_op[nq]);
            }
            ref_prev[q] = ref_next[q] = NONE;
        }
        op_st[o] = OP_DONE;
        map_need[op_map[o]] -= MAX_CREATES[op_kind[o]];
    }
    void splice(uint32_t o)
    {
        splice_core(o, [&](uint32_t x) { release(x); });
        --pending;
    }
    // one row of cv_epnode_receive (rel / done: as splice_core, the pending count's share)
    template <class R>
    int receive_row(uint32_t i, uint32_t ep, uint8_t has, int32_t &op, R &&rel, uint64_t &done)
    {
        if (i >= n || dl_first[i] == NONE) return -EPROTO;
        uint32_t o = dl_first[i], k = 0;
        while (k < dl_cnt[i] && op_map[o] >> 1 != ep) ++k, ++o;
        if (k == dl_cnt[i] || op_st[o] != OP_PENDING) return -EPROTO;
        // a record: the delivery runs once nothing earlier on its keys waits; none: nothing
        // runs here -- it leaves its keys' lists now (its successors wait for its pending
        // predecessors instead), or, on a chained map, runs as a no-op in its turn
        op = has ? (int32_t)o : -1;
        if (has) {
            op_st[o] = OP_RESOLVED;
        } else if (map_chain[op_map[o]]) {
            op_st[o] = OP_NOOP;
        } else {
            splice_core(o, rel);
            ++done;
        }
        return 0;
    }
    int room(bool first);
    // the operations of `kind` that can run now (deliveries: with their record), and
    // those they free in turn, in packet order.  Level by level: a large level is
    // finished on host threads, each taking the operations of its maps (an operation's
    // successors are in its map: no shared count), a small one in place.
    void run_ready(int kind, std::vector<uint32_t> &out)
    {
        std::vector<uint32_t> keep, cur, &z = zero[kind];
        auto sift = [&](std::vector<uint32_t> &from) {       // runnable ones to cur, the rest kept
            for (uint32_t o : from) {
                if (op_st[o] == OP_DONE) continue;
                if (op_st[o] == OP_PENDING) keep.push_back(o);  // (a delivery whose record has not arrived)
                else cur.push_back(o);
            }
            from.clear();
        };
        sift(z);
        const uint32_t T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        static const bool tm = getenv("CV_EPNODE_TIMES") != nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t levels = 0, big = 0;
        const size_t first = cur.size();
        while (!cur.empty()) {
            ++levels;
            std::vector<uint32_t> lvl;
            lvl.swap(cur);
            if (lvl.size() < 8192 || T == 1) {
                for (uint32_t o : lvl) {
                    if (op_st[o] == OP_RESOLVED) out.push_back(o);   // (OP_NOOP: not delivered here, nothing to run)
                    finish(o);
                }
                sift(z);
                continue;
            }
            ++big;
            std::vector<std::vector<uint32_t>> rel(2 * T), outs(T);
            std::vector<uint64_t> done(T, 0);
            std::vector<std::thread> th;
            for (uint32_t t = 0; t < T; ++t)
                th.emplace_back([&, t] {                      // (thread t: the level's operations of its maps)
                    auto push = [&](uint32_t x) {
                        if (--op_wait[x] == 0) rel[2 * t + op_kind[x]].push_back(x);
                    };
                    for (const uint32_t o : lvl) {
                        if (op_map[o] % T != t) continue;
                        if (op_st[o] == OP_RESOLVED) outs[t].push_back(o);
                        finish_core(o, push);
                        ++done[t];
                    }
                });
            for (auto &x : th) x.join();
            for (uint32_t t = 0; t < T; ++t) {
                out.insert(out.end(), outs[t].begin(), outs[t].end());
                pending -= done[t];
                zero[1 - kind].insert(zero[1 - kind].end(), rel[2 * t + 1 - kind].begin(), rel[2 * t + 1 - kind].end());
                z.insert(z.end(), rel[2 * t + kind].begin(), rel[2 * t + kind].end());
            }
            sift(z);
        }
        z.swap(keep);
        if (tm)
            fprintf(stderr, "[epnode run] kind %d: %zu first, %zu out, %u levels (%u threaded), %.1f ms\n", kind, first,
                    out.size(), levels, big,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        // in operation order, which is packet order (a flag pass when the round is large)
        if (out.size() * 16 < op_pkt.size()) {
            std::sort(out.begin(), out.end());
        } else {
            std::vector<uint8_t> f(op_pkt.size(), 0);
            for (uint32_t o : out) f[o] = 1;
            size_t j = 0;
            for (uint32_t o = 0; o < (uint32_t)f.size(); ++o)
                if (f[o]) out[j++] = o;
        }
    }
};

// live + the creates the pending operations may make > max_entries: the map may fill.
// First round: every map's room; chain the maps that may fill.  Later: the chained maps'
// room again; a map with room for every create its operations may still make leaves
// the chain (live + need never grows: an operation adds at most what it took from need).
int cv_epnode::room(bool first)
{
    std::vector<int> hs;
    std::vector<uint32_t> ms;
    for (uint32_t m : active)
        if (map_handle[m] >= 0 && (first || map_chain[m])) {
            hs.push_back(map_handle[m]);
            ms.push_back(m);
        }
    if (hs.empty()) return 0;
    std::vector<uint64_t> live(hs.size()), cap(hs.size());
    const int r = counts ? counts(counts_arg, hs.data(), (uint32_t)hs.size(), live.data(), cap.data())
                         : cv::ct_counts(ctx, hs, live, cap);
    if (r) return r;
    for (size_t k = 0; k < ms.size(); ++k) {
        const uint32_t m = ms[k];
        const bool tight = (int64_t)live[k] + std::max<int64_t>(map_need[m], 0) > (int64_t)cap[k];
        uint32_t &h = map_head[m];
        while (h < map_off[m + 1] && op_st[map_ops[h]] == OP_DONE) ++h;
        if (first && tight) {                                 // every operation after the first waits
            map_chain[m] = 1;
            chained0++;
            for (uint32_t j = map_off[m] + 1; j < map_off[m + 1]; ++j) op_wait[map_ops[j]]++;
        } else if (!first && !tight && map_chain[m]) {        // out of the chain: drop the links still counted
            map_chain[m] = 0;
            for (uint32_t j = std::max(h, map_off[m] + 1); j < map_off[m + 1]; ++j)
                if (op_st[map_ops[j - 1]] != OP_DONE && op_st[map_ops[j]] != OP_DONE) release(map_ops[j]);
        }
    }
    return 0;
}

extern "C" {

int cv_epnode_open(cv_ctx *ctx, uint32_t rank, uint32_t world, const uint8_t *frames, uint32_t stride, uint32_t n,
                   const uint16_t *src_ep, cv_epnode **out)
{
    if (!ctx || !out || !world || rank >= world || (n && (!frames || !src_ep)) || stride < 54) return -EINVAL;
    const bool tm = getenv("CV_EPNODE_TIMES") != nullptr;
    auto t_0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!tm) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[epnode open] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t_0).count());
        t_0 = t;
    };
    int r = 0;
    const std::shared_ptr<const NodeIdx> ix = node_index(ctx, r);
    if (!ix) return r;
    const cv::NodeView &v = ix->v;
    const uint32_t ne = (uint32_t)v.eps.size();
    const Csr<uint32_t> &where = ix->where;
    const Csr<uint64_t> &backends = ix->backends;
    const Csr<VipPort> &vips = ix->vips;
    const uint64_t lob = ix->lob;
    lap("node view and indexes");
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
    // per packet: candidates, peers and operations, over packet ranges on host threads
    // (each range its own buffers, joined in packet order)
    struct Part {
        std::vector<uint32_t> cand, cand_n, op_pkt, op_map, op_np;
        std::vector<uint8_t> op_kind;
        std::vector<uint64_t> peer;
        uint64_t n_src = 0, n_dl = 0;
        int err = 0;
        void swap_out(Part &o) { std::swap(cand, o.cand); std::swap(peer, o.peer); }   // (frees o's big arrays)
    };
    const uint32_t T = n < (1u << 14) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<Part> parts(T);
    auto build = [&](uint32_t t, uint32_t i0, uint32_t i1) {
        Part &P = parts[t];
        std::vector<uint32_t> c;
        std::vector<uint64_t> sp, dp;
        for (uint32_t i = i0; i < i1; ++i) {
            const uint8_t *f = frames + (size_t)i * stride;
            const uint32_t s = src_ep[i];
            if (s >= ne) { P.err = -EINVAL; return; }
            c.clear();
            sp.clear();
            dp.clear();
            const bool is4 = f[12] == 0x08 && f[13] == 0x00, is6 = f[12] == 0x86 && f[13] == 0xDD;
            nd->v6[i] = is6;
            if (is4 || is6) {
                const uint64_t sa = ahash(is4 ? addr4(f + 26) : addr6(f + 22)), da = ahash(is4 ? addr4(f + 30) : addr6(f + 38));
                const auto bes = backends.find(da);
                auto add_where = [&](uint64_t a) {
                    const auto w = where.find(a);
                    c.insert(c.end(), where.val.begin() + w.first, where.val.begin() + w.second);
                };
                add_where(da);
                bool loop = false;
                for (uint32_t k = bes.first; k < bes.second; ++k) {
                    add_where(backends.val[k]);
                    loop |= backends.val[k] == sa;
                }
                std::sort(c.begin(), c.end());
                c.erase(std::unique(c.begin(), c.end()), c.end());
                // peers: the source program's -- the destination, a VIP's backends, and the
                // loopback address when the client backs the VIP itself; the delivery's -- the
                // source as the source program left it: itself, a VIP it backs (reverse NAT of
                // a reply), or the loopback address
                loop = loop && v.loopback;
                sp.push_back(da);
                sp.insert(sp.end(), backends.val.begin() + bes.first, backends.val.begin() + bes.second);
                dp.push_back(sa);
                // a TCP / UDP reply is reverse-NATed only by a connection whose translated
                // dport is its sport (lb4_xlate / lb6_xlate: the backend's port, else the
                // original dport -- the VIP's for an L4 service); ICMP (RELATED) or an
                // unparsed header: any VIP the source backs
                uint32_t sport = 0;
                bool ports = false;
                if (is4) {
                    const uint32_t pr = f[23], off = 14 + 4 * (f[14] & 0xFu);
                    ports = (pr == 6 || pr == 17) && off + 2 <= stride;
                    if (ports) sport = f[off] | f[off + 1] << 8;
                } else {
                    ports = (f[20] == 6 || f[20] == 17) && 56 <= stride;
                    if (ports) sport = f[54] | f[55] << 8;
                }
                const auto vi = vips.find(sa);
                for (uint32_t k = vi.first; k < vi.second; ++k) {
                    const VipPort &x = vips.val[k];
                    if (!ports || (x.bport ? x.bport == sport : (!x.vport || x.vport == sport))) dp.push_back(x.vip);
                }
                if (loop) {
                    sp.push_back(lob);
                    dp.push_back(lob);
                }
            }
            if (c.size() > 255) { P.err = -E2BIG; return; }          // (dl_cnt is a byte)
            P.cand.insert(P.cand.end(), c.begin(), c.end());
            P.cand_n.push_back((uint32_t)c.size());
            const uint32_t fam = is6 ? 1 : 0;
            auto add_op = [&](uint32_t kind, uint32_t ep, const std::vector<uint64_t> &ps) {
                P.op_pkt.push_back(i);
                P.op_kind.push_back((uint8_t)kind);
                P.op_map.push_back(ep * 2 + fam);
                P.peer.insert(P.peer.end(), ps.begin(), ps.end());
                P.op_np.push_back((uint32_t)ps.size());
            };
            if (nd->owned(s)) {
                add_op(0, s, sp);
                P.n_src++;
            }
            for (uint32_t d : c)
                if (nd->owned(d)) {
                    add_op(1, d, dp);
                    P.n_dl++;
                }
        }
    };
    {
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < T; ++t)
            th.emplace_back(build, t, (uint32_t)((uint64_t)n * t / T), (uint32_t)((uint64_t)n * (t + 1) / T));
        for (auto &x : th) x.join();
    }
    lap("per-packet build");
    std::vector<uint64_t> peer64;                                 // (the operations' peers, as hashes)
    {
        // the parts joined in packet order: offsets first, then every part copies itself
        std::vector<size_t> co(T + 1, 0), oo(T + 1, 0), po(T + 1, 0);
        std::vector<uint32_t> io(T + 1, 0);
        for (uint32_t t = 0; t < T; ++t) {
            const Part &P = parts[t];
            if (P.err) return P.err;
            co[t + 1] = co[t] + P.cand.size();
            oo[t + 1] = oo[t] + P.op_pkt.size();
            po[t + 1] = po[t] + P.peer.size();
            io[t + 1] = io[t] + (uint32_t)P.cand_n.size();
            nd->n_src += P.n_src;
            nd->n_dl += P.n_dl;
        }
        if (po[T] >= 0xFFFFFFFFull || co[T] >= 0xFFFFFFFFull) return -E2BIG;
        nd->cand.resize(co[T]);
        nd->op_pkt.resize(oo[T]);
        nd->op_kind.resize(oo[T]);
        nd->op_map.resize(oo[T]);
        nd->op_poff.resize(oo[T] + 1);
        peer64.resize(po[T]);
        auto join = [&](uint32_t t) {
            Part &P = parts[t];
            std::copy(P.cand.begin(), P.cand.end(), nd->cand.begin() + co[t]);
            uint32_t c = (uint32_t)co[t];
            for (size_t k = 0; k < P.cand_n.size(); ++k) {
                nd->cand_off[io[t] + k] = c;
                c += P.cand_n[k];
            }
            uint32_t q = (uint32_t)po[t];
            for (size_t k = 0; k < P.op_pkt.size(); ++k) {
                const uint32_t o = (uint32_t)(oo[t] + k), pk = P.op_pkt[k];
                if (P.op_kind[k] == 1) {
                    if (nd->dl_first[pk] == ~0u) nd->dl_first[pk] = o;
                    nd->dl_cnt[pk]++;
                }
                nd->op_pkt[o] = pk;
                nd->op_kind[o] = P.op_kind[k];
                nd->op_map[o] = P.op_map[k];
                nd->op_poff[o] = q;
                q += P.op_np[k];
            }
            std::copy(P.peer.begin(), P.peer.end(), peer64.begin() + po[t]);
            Part().swap_out(P);
        };
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < T; ++t) th.emplace_back(join, t);
        for (auto &x : th) x.join();
        nd->cand_off[n] = (uint32_t)co[T];
        nd->op_poff[oo[T]] = (uint32_t)po[T];
    }
    lap("join");
    const uint32_t nops = (uint32_t)nd->op_pkt.size(), nm = ne * 2;
    nd->pending = nops;
    // per map, its operations in order: a stable counting sort by map over operation ranges
    // on host threads (each range counts, the counts are scanned map by map and range by
    // range, each range places its operations); with it each operation's state and its key
    // references' owner
    nd->op_st.resize(nops);
    nd->map_ops.resize(nops);
    nd->op_mpos.resize(nops);
    nd->ref_op.resize(peer64.size());
    nd->ref_next.assign(peer64.size(), cv_epnode::NONE);
    nd->ref_prev.assign(peer64.size(), cv_epnode::NONE);
    {
        const uint32_t T = nops < (1u << 16) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::vector<uint32_t>> at(T, std::vector<uint32_t>(nm, 0));
        auto range = [&](uint32_t t) {
            return std::make_pair((uint32_t)((uint64_t)nops * t / T), (uint32_t)((uint64_t)nops * (t + 1) / T));
        };
        auto par = [&](auto &&f) {
            std::vector<std::thread> th;
            for (uint32_t t = 0; t < T; ++t) th.emplace_back(f, t);
            for (auto &x : th) x.join();
        };
        par([&](uint32_t t) {
            const auto r = range(t);
            for (uint32_t o = r.first; o < r.second; ++o) {
                nd->op_st[o] = nd->op_kind[o] == 0 ? OP_RESOLVED : OP_PENDING;   // (a source program needs no record)
                at[t][nd->op_map[o]]++;
                for (uint32_t q = nd->op_poff[o]; q < nd->op_poff[o + 1]; ++q) nd->ref_op[q] = o;
            }
        });
        nd->map_off.assign(nm + 1, 0);
        uint32_t run = 0;
        for (uint32_t m = 0; m < nm; ++m) {
            nd->map_off[m] = run;
            for (uint32_t t = 0; t < T; ++t) {
                const uint32_t c = at[t][m];
                at[t][m] = run;
                run += c;
            }
        }
        nd->map_off[nm] = run;
        par([&](uint32_t t) {
            const auto r = range(t);
            for (uint32_t o = r.first; o < r.second; ++o) {
                const uint32_t k = at[t][nd->op_map[o]]++;
                nd->map_ops[k] = o;
                nd->op_mpos[o] = k;
            }
        });
    }
    nd->map_head.assign(nd->map_off.begin(), nd->map_off.end() - 1);
    lap("map order");
    nd->op_wait.assign(nops, 0);
    {
        const std::vector<uint32_t> &ref_op = nd->ref_op;
        // maps are independent: their links are built on host threads, each with its
        // maps' share of the wait counts (an operation is in one map)
        // per map one pass over its references in operation order (= packet order) with a
        // small open-addressing table peer -> the last reference on it: each reference
        // links to that one (the same links as sorting the (peer, reference) pairs)
        auto link = [&](uint32_t m0, uint32_t m1) {
            std::vector<uint64_t> tk;                             // (peer, or 0: empty)
            std::vector<uint32_t> tv;                             // (its last reference)
            std::vector<uint32_t> used;
            for (uint32_t m = m0; m < m1; ++m) {
                size_t refs = 0;
                for (uint32_t k = nd->map_off[m]; k < nd->map_off[m + 1]; ++k) {
                    const uint32_t o = nd->map_ops[k];
                    refs += nd->op_poff[o + 1] - nd->op_poff[o];
                }
                if (!refs) continue;
                size_t cap = 64;
                while (cap < 2 * refs) cap <<= 1;
                if (tk.size() < cap) {
                    tk.assign(cap, 0);
                    tv.assign(cap, 0);
                    used.clear();
                }
                const uint64_t mask = cap - 1;
                for (uint32_t k = nd->map_off[m]; k < nd->map_off[m + 1]; ++k) {
                    const uint32_t o = nd->map_ops[k];
                    for (uint32_t q = nd->op_poff[o]; q < nd->op_poff[o + 1]; ++q) {
                        const uint64_t pe = peer64[q];            // (ahash: never 0)
                        uint64_t h = (pe ^ (pe >> 29)) & mask;
                        while (tk[h] && tk[h] != pe) h = (h + 1) & mask;
                        if (!tk[h]) {
                            tk[h] = pe;
                            used.push_back((uint32_t)h);
                        } else {
                            const uint32_t pq = tv[h], a = ref_op[pq];
                            if (a != o) {                         // (a peer named twice by one operation links once)
                                nd->ref_next[pq] = q;             // (o waits for a on this peer)
                                nd->ref_prev[q] = pq;
                                nd->op_wait[o]++;
                            }
                        }
                        tv[h] = q;
                    }
                }
                for (uint32_t h : used) tk[h] = 0;                // (only the slots this map took)
                used.clear();
            }
        };
        const uint32_t T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < T; ++t) th.emplace_back(link, (uint32_t)((uint64_t)nm * t / T), (uint32_t)((uint64_t)nm * (t + 1) / T));
        for (auto &x : th) x.join();
    }
    lap("links");
    nd->map_handle.assign(nm, -1);
    nd->map_need.assign(nm, 0);
    nd->map_chain.assign(nm, 0);
    for (uint32_t m = 0; m < nm; ++m) {
        if (nd->map_off[m + 1] == nd->map_off[m]) continue;
        nd->active.push_back(m);
        nd->map_handle[m] = (m & 1) ? v.eps[m >> 1].ct6 : v.eps[m >> 1].ct4;
    }
    for (uint32_t o = 0; o < nops; ++o) nd->map_need[nd->op_map[o]] += MAX_CREATES[nd->op_kind[o]];
    lap("maps");
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
    for (uint32_t m : nd->active) t += nd->map_chain[m];
    stats[0] = nd->rounds;
    stats[1] = nd->n_src;
    stats[2] = nd->n_dl;
    stats[3] = nd->chained0;
    stats[4] = t;
    stats[5] = nd->sent;
    return 0;
}

int cv_epnode_sources(cv_epnode *nd, uint32_t *pkts, uint32_t cap)
{
    if (!nd || (cap && !pkts)) return -EINVAL;
    int r;
    if (!nd->rounds++) {                                   // every map's room, once; then who waits for nothing
        if ((r = nd->room(true))) return r;
        for (uint32_t o = 0; o < (uint32_t)nd->op_pkt.size(); ++o)
            if (!nd->op_wait[o]) nd->zero[nd->op_kind[o]].push_back(o);
    } else {
        bool any = false;
        for (uint32_t m : nd->active) any |= nd->map_chain[m] != 0;
        if (any && (r = nd->room(false))) return r;        // (room re-read for the maps that may fill)
    }
    std::vector<uint32_t> out;
    nd->run_ready(0, out);
    if (out.size() > cap) return -ENOSPC;
    for (size_t j = 0; j < out.size(); ++j) pkts[j] = nd->op_pkt[out[j]];
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
    const uint32_t T = n < (1u << 16) ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (T == 1) {
        uint64_t done = 0;
        for (uint32_t j = 0; j < n; ++j) {
            const int r = nd->receive_row(row_pkt[j], row_ep[j], row_has[j], op[j],
                                          [&](uint32_t x) { nd->release(x); }, done);
            nd->pending -= done;
            done = 0;
            if (r) return r;
        }
        return 0;
    }
    // a row changes only its destination's maps: the rows split by endpoint over host
    // threads, each with its own lists of what becomes free
    std::vector<std::vector<uint32_t>> rel(2 * T);
    std::vector<uint64_t> done(T, 0);
    std::vector<int> err(T, 0);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            auto push = [&](uint32_t x) {
                if (--nd->op_wait[x] == 0) rel[2 * t + nd->op_kind[x]].push_back(x);
            };
            for (uint32_t j = 0; j < n; ++j) {
                if (row_ep[j] % T != t) continue;
                if ((err[t] = nd->receive_row(row_pkt[j], row_ep[j], row_has[j], op[j], push, done[t]))) return;
            }
        });
    for (auto &x : th) x.join();
    for (uint32_t t = 0; t < T; ++t) {
        nd->pending -= done[t];
        for (int k = 0; k < 2; ++k) nd->zero[k].insert(nd->zero[k].end(), rel[2 * t + k].begin(), rel[2 * t + k].end());
    }
    for (uint32_t t = 0; t < T; ++t)
        if (err[t]) return err[t];
    return 0;
}

int cv_epnode_deliveries(cv_epnode *nd, uint32_t *ops, uint32_t *pkts, uint32_t cap)
{
    if (!nd || (cap && (!ops || !pkts))) return -EINVAL;
    std::vector<uint32_t> out;
    nd->run_ready(1, out);
    if (out.size() > cap) return -ENOSPC;
    for (size_t j = 0; j < out.size(); ++j) {
        ops[j] = out[j];
        pkts[j] = nd->op_pkt[out[j]];
    }
    return (int)out.size();
}

}  // extern "C"
