// cv_ctx.cpp — the C-ABI (include/cilium_hip.h): map store, program->map binding,
// compilation of the device tables and the batch entry points.
//
// Maps: every map the agent creates lives in a HostMap with the kernel's semantics
// (pkg/bpf/bpf.go:101-245 -> kernel/bpf).  Maps the datapath reads are compiled into
// per-role device tables (cv_hash.hpp, cv_lpm.hpp) at the next batch boundary
// (cv_sync).  Two kinds of state are written by the datapath itself and are
// device-authoritative: policy counters (policy.h:76-100) and conntrack tables
// (conntrack.h); host reads of them fetch from HBM.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/cilium_hip.h"
#include "cv_dp.hpp"
#include "cv_hostmap.hpp"
#include "cv_node.hpp"

using namespace cv;

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    int alloc(size_t bytes)
    {
        release();
        if (!bytes) return 0;
        if (hipMalloc(&p, bytes) != hipSuccess) { p = nullptr; return -ENOMEM; }
        n = bytes;
        return 0;
    }
    int upload(const void *src, size_t bytes)
    {
        int r = alloc(bytes);
        if (r) return r;
        return hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -EIO;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// A device hash table plus the host image it was built from.
struct DevHash {
    DevBuf buckets, vals, aux;
    std::vector<uint32_t> hb;   // host image of the buckets
    HashTable view{};
    uint64_t nb = 0;
};

template <class S>
int build_hash(DevHash &d, const std::vector<std::vector<uint32_t>> &keys, const std::vector<std::vector<uint32_t>> &ivals,
               uint32_t vstride, const std::vector<uint8_t> *vals, std::vector<int64_t> *slots, size_t room = 0)
{
    uint64_t nb = buckets_for(keys.size() + room, S::SPB);   // (room: entries later writes may add in place)
    for (int attempt = 0; attempt < 8; ++attempt, nb <<= 1) {
        d.hb.assign(nb * S::BW, 0);
        HashTable t{d.hb.data(), nullptr, nb - 1, vstride, (uint32_t)S::SPB};
        bool ok = true;
        if (slots) slots->assign(keys.size(), -1);
        for (size_t i = 0; i < keys.size() && ok; ++i) {
            int64_t s = host_upsert<S>(t, keys[i].data(), (S::IVW || S::IVH) ? ivals[i].data() : nullptr);
            if (s < 0) ok = false;
            else if (slots) (*slots)[i] = s;
        }
        if (!ok) continue;
        d.nb = nb;
        int r = d.buckets.upload(d.hb.data(), d.hb.size() * 4);
        if (r) return r;
        if (vstride) {
            std::vector<uint8_t> hv(nb * S::SPB * vstride, 0);
            if (vals && slots)
                for (size_t i = 0; i < keys.size(); ++i)
                    memcpy(&hv[(size_t)(*slots)[i] * vstride], vals->data() + i * vstride, vstride);
            r = d.vals.upload(hv.data(), hv.size());
            if (r) return r;
        } else {
            d.vals.release();
        }
        d.view = HashTable{d.buckets.as<uint32_t>(), d.vals.as<uint8_t>(), nb - 1, vstride, (uint32_t)S::SPB};
        return 0;
    }
    return -E2BIG;
}

struct Pfx {
    uint32_t prio;       // full prefixlen in the map
    int plen;            // prefix length within the address
    uint32_t a[4];       // address words (raw network order)
    uint32_t value;
};

struct DevLpm4 {
    DevBuf l1, chunks;
    DevHash full;              // the /32 prefixes (hash front of the trie)
    Lpm4 view{nullptr, nullptr, HashTable{}};
    // host image for incremental updates (ipcache): the trie as built, the device
    // chunk capacity, the /17-/31 prefixes per level-1 slot, the map it mirrors
    bool image = false;
    Lpm4Builder hb;
    size_t chunk_cap = 0, chunks_on_dev = 0;
    std::unordered_map<uint32_t, std::vector<Pfx>> longer;
    const void *of = nullptr;
    uint64_t front_live = 0;
};

struct DevLpm6 {
    DevHash h;
    DevBuf lens;                 // LENS_CAP bytes: the distinct prefix lengths, descending
    Lpm6 view{};
    // host side for incremental updates (ipcache): live entries, entries per length
    uint64_t live = 0;
    std::map<int, uint32_t> lens_cnt;
};
constexpr size_t LENS_CAP = 160;

enum MapKind { MK_PLAIN = 0, MK_CT4 = 1, MK_CT6 = 2 };

struct MapObj {
    std::unique_ptr<HostMap> hm;
    int kind = MK_PLAIN;
    // policy compilation (when bound as an endpoint policy map)
    bool is_policy = false;
    DevHash pol;
    uint64_t pol_version = 0;
    uint64_t pol_live = 0;              // live keys in the compiled table
    std::set<std::string> written;      // keys whose value the agent wrote since the last sync
    // conntrack (device-authoritative)
    DevHash ct;
    uint32_t ct_id = 0;
    DevBuf live;                        // u64 live-entry count on the device (HashTable::live)
    uint64_t live_upper = 0;            // an upper bound of it the host plans launches with
    uint64_t cap = 0;                   // max_entries
    uint64_t gen = 0;                   // bumped by every device write: batches, map API, GC
    // GetNextKey walk over the device table: its entries in slot order as of `gen`
    uint64_t snap_gen = ~0ull;
    std::vector<uint8_t> snap_keys;
    size_t snap_last = ~(size_t)0;                     // position of the key the last call returned
    std::unordered_map<std::string, size_t> snap_index;   // built only for walks that jump
};

struct Endpoint {
    uint16_t lxc_id;
    uint32_t seclabel;
    int policy, ct4;
    int ct6 = -1;
    uint32_t ipv4 = 0;         // LXC_IPV4 (raw); set by cv_endpoint_config
    uint32_t ipv6[4] = {0, 0, 0, 0};
    uint32_t mac[2] = {0, 0}, node_mac[2] = {0, 0};
};

// Stream-ordered publication of the agent's incremental table writes: the changed
// words are gathered on the host while the writes are applied to the host images, then
// at the batch boundary one pinned staging buffer goes to the device (one async copy)
// and k_patch writes every run of words into its table, in the stream of the batch
// about to run: batches already submitted see the old words, later ones the new --
// the kernel's RCU per-element visibility at batch granularity, without waiting for
// the device.
struct PatchQueue {
    std::vector<PatchRec> recs;
    std::vector<uint32_t> words;
    void add(void *dst, const void *src, size_t nwords)
    {
        if (!nwords) return;
        recs.push_back(PatchRec{reinterpret_cast<unsigned long long>(dst), (uint32_t)nwords, (uint32_t)words.size()});
        const uint32_t *w = static_cast<const uint32_t *>(src);
        words.insert(words.end(), w, w + nwords);
    }
    size_t mark() const { return recs.size(); }
    void undo(size_t m)                        // (a role falling back to a full compile)
    {
        if (m >= recs.size()) return;
        words.resize(recs[m].src);
        recs.resize(m);
    }
};

struct Staging {                               // pinned host + device staging of one publication
    void *host = nullptr, *dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;                 // recorded after its k_patch
};

}  // namespace

// Test and measurement hooks, read once when the context opens (never per launch).
// CV_SNAP_ABLATE is a timing-only ablation that makes undone egress passes wrong; it is
// honoured only together with CV_TIMING_ONLY=1.
struct Hooks {
    bool coarse_groups = false;    // CV_COARSE_GROUPS: 8-bit group keys (merged runs, tests)
    bool no_uni = false;           // CV_NO_UNI4: per-packet endpoint lines (tests)
    bool eam_force = false;        // CV_EAM_FORCE: the many-map egress admission on one map (measurements)
    bool egress_guarded = false;   // CV_EGRESS_GUARDED: planned launches instead of admission (tests)
    bool snap_ablate = false;      // CV_SNAP_ABLATE + CV_TIMING_ONLY: no slot saved (timing only)
    int eadm_max_passes = 8;       // CV_EADM_MAX_PASSES (tests of the fallback)
    void read()
    {
        coarse_groups = getenv("CV_COARSE_GROUPS") != nullptr;
        no_uni = getenv("CV_NO_UNI4") != nullptr;
        eam_force = getenv("CV_EAM_FORCE") != nullptr;
        egress_guarded = getenv("CV_EGRESS_GUARDED") != nullptr;
        const char *t = getenv("CV_TIMING_ONLY");
        snap_ablate = getenv("CV_SNAP_ABLATE") && t && !strcmp(t, "1");
        const char *mp = getenv("CV_EADM_MAX_PASSES");
        eadm_max_passes = mp && atoi(mp) >= 1 && atoi(mp) <= 64 ? atoi(mp) : 8;
    }
};

struct cv_ctx {
    int device = 0;
    Hooks hk;
    uint32_t flags = CV_F_DEFAULT;
    std::mutex mu;
    std::vector<std::unique_ptr<MapObj>> maps;
    int role[CV_NUM_ROLES];
    uint64_t role_version[CV_NUM_ROLES];
    DevHash cidr4_fix, cidr6_fix, lxc4, lxc6;
    DevLpm4 cidr4_dyn, ipc4;
    DevLpm6 cidr6_dyn, ipc6;
    DevHash lb4, lb6;
    DevBuf revnat4, revnat6;
    cv_node_cfg node{};
    std::vector<Endpoint> eps;
    bool eps_dirty = true;
    uint64_t eps_gen = 0;      // bumped by every endpoint change (map_table's cache key)
    uint64_t uid = 0;          // unique per cv_open in the process (caches keyed by context)
    DevBuf eps_dev, ephot_dev, ephot6_dev, ep_of_lxc;
    bool uni4_on = false;      // every endpoint on one policy + CT4 map, LXC_IPV4 set (DpParams::uni4)
    bool uni6_on = false;      // every endpoint on one policy + CT6 map (DpParams::uni6)
    EpHot uni4{}, uni6{};
    DevBuf metrics_own;
    unsigned long long *metrics = nullptr;
    DevBuf gtable, gsingle, gslot, gnext, gsrec, gparent, geg, gorder, gcursor, gqueue, gwork, gifx;
    DevBuf gdel, gest;            // egress: local-delivery records (DEL_SLOTS x 16 B per packet),
                                  // the conntrack stage's input states (64 B per packet)
    DevBuf gres, gdel_ev;         // egress: packed outputs (16 B), delivery records' event part (32 B)
    DevBuf gpkey, gent, gbig, gcnt, gwork6, ghword, ghcnt;   // the netdev path's binned grouping
    DevBuf gsjob;                 // (its split-key jobs)
    DevBuf gbx;                   // (its big-bin records)
    DevBuf ghot;                  // elephants in parallel (k_hpar_*)
    DevBuf adm_ib, adm_tsum, adm_win;  // conntrack admission next to max_entries
    DevBuf adm_mi, adm_keys, adm_sort; // (per packet: map index; walk keys, sorted; radix-sort scratch)
    DevBuf adm_evt;                    // (k_ct_intent's spill tables)
    uint32_t adm_stamp = 0;
    // the launch's CT maps as admission and the live-count reads see them (map_table)
    std::vector<MapObj *> mt_maps;
    uint64_t mt_eps = ~(uint64_t)0;   // (eps_gen the table was built at)
    DevBuf mt_live, mt_cap, mt_epmi4, mt_epmi6, mt_out;
    DevBuf bnd_buf;                    // the room check's per-map bounds, per-LB-slot counts, flags (CtBound)
    uint64_t bound_checks = 0, bound_fits = 0;
    DevBuf eadm_save, eadm_buf;        // egress admission: the state a pass writes, intents + budgets
    DevBuf eam_buf, eam_keys, eam_snap;  // (many CT maps: per-slot intents + budgets, walk keys, the slot set)
    Snap eam_snap_host[2]{};
    uint64_t gcap = 0, gn = 0;
    bool g_egress = false;     // parent + egress scratch allocated
    uint32_t epoch = 0;
    uint32_t serial = 0;       // launches so far (GroupScratch::serial)
    DevBuf ctio;
    uint32_t next_ct_id = 1;
    uint32_t chunk = MAX_CHUNK;    // packets per launch (CV_MAX_CHUNK env may lower it, tests)
    // drop notification ring (cv_notify_attach), device pointers
    cv_drop_notify *notify = nullptr;
    uint32_t notify_cap = 0;
    uint32_t *notify_count = nullptr;
    // trace notification ring (cv_trace_attach)
    cv_trace_notify *trace = nullptr;
    uint32_t trace_cap = 0, trace_agg = 0, ingress_ifindex = 0;
    uint32_t *trace_count = nullptr;
    // table publication (PatchQueue) and batch ordering across streams
    PatchQueue pq;
    std::vector<Staging> staging;
    hipEvent_t last_ev = nullptr;              // the last batch's (or publication's) completion
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    bool force_full = false;                   // a publication was lost: compile ipcache / policies in full
    uint64_t publications = 0, full_compiles = 0;
    // the walkers' error word (GroupScratch::err): host-mapped, so a corrupt list a kernel
    // met fails the context's next call with -EPROTO without a device wait
    uint32_t *gerr_host = nullptr, *gerr_dev = nullptr;
};

namespace {

MapObj *get(cv_ctx *c, int h)
{
    if (h < 0 || (size_t)h >= c->maps.size()) return nullptr;
    return c->maps[h].get();
}

int set_device(cv_ctx *c)
{
    if (c->device < 0) return -ENODEV;      // host-only context
    return hipSetDevice(c->device) == hipSuccess ? 0 : -ENODEV;
}

std::string kstr(const uint8_t *k, uint32_t n) { return std::string(reinterpret_cast<const char *>(k), n); }

inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

// ---------------------------------------------------------------- role compilers
int compile_lxc(cv_ctx *c, HostMap *m)
{
    std::vector<std::vector<uint32_t>> k4, v4, k6, v6;
    // 16-B side values per entry: endpoint_info.ifindex, .mac, .node_mac (common.h:165-173)
    std::vector<uint8_t> if4, if6;
    auto side = [](std::vector<uint8_t> &o, const uint8_t *v) {
        o.insert(o.end(), v, v + 4);
        o.insert(o.end(), v + 16, v + 22);
        o.insert(o.end(), v + 24, v + 30);
    };
    if (m) {
        if (m->ks != 20 || m->vs < 12) return -EINVAL;
        m->for_each([&](const uint8_t *k, const uint8_t *v) {
            if (k[17] || k[18] || k[19]) return;            // pads are zero in datapath keys
            const uint32_t iv = rd16(v + 6) | ((rd32(v + 8) & 1u) << 16) | ((rd32(v) != 0) << 17);
            if (k[16] == 1) {
                for (int i = 4; i < 16; ++i) if (k[i]) return;
                k4.push_back({rd32(k)});
                v4.push_back({iv});
                side(if4, v);
            } else if (k[16] == 2) {
                k6.push_back({rd32(k), rd32(k + 4), rd32(k + 8), rd32(k + 12)});
                v6.push_back({iv});
                side(if6, v);
            }
        });
    }
    std::vector<int64_t> s4, s6;
    int r = build_hash<LxcV4Spec>(c->lxc4, k4, v4, 16, &if4, &s4);
    if (!r) r = build_hash<LxcV6Spec>(c->lxc6, k6, v6, 16, &if6, &s6);
    if (!m) { c->lxc4.view = HashTable{}; c->lxc6.view = HashTable{}; }
    return r;
}

int compile_cidr_fix(cv_ctx *c, HostMap *m, bool v6)
{
    std::vector<std::vector<uint32_t>> keys, none;
    DevHash &d = v6 ? c->cidr6_fix : c->cidr4_fix;
    if (!m) { d.view = HashTable{}; return 0; }
    if (m->ks != (v6 ? 20u : 8u)) return -EINVAL;
    m->for_each([&](const uint8_t *k, const uint8_t *) {
        if (rd32(k) != (v6 ? 128u : 32u)) return;           // datapath keys carry prefixlen 32/128
        if (v6) keys.push_back({rd32(k + 4), rd32(k + 8), rd32(k + 12), rd32(k + 16)});
        else keys.push_back({rd32(k + 4)});
    });
    return v6 ? build_hash<Cidr6Spec>(d, keys, none, 0, nullptr, nullptr)
              : build_hash<Cidr4Spec>(d, keys, none, 0, nullptr, nullptr);
}

// `image`: keep the host trie and the /17-/31 index so later writes can be applied
// incrementally (update_ipcache4), with device room for that many more chunks
int upload_lpm4(DevLpm4 &d, std::vector<Pfx> &px, bool image = false)
{
    std::stable_sort(px.begin(), px.end(), [](const Pfx &x, const Pfx &y) { return x.prio < y.prio; });
    Lpm4Builder b;
    std::vector<std::vector<uint32_t>> k32, v32;
    d.longer.clear();
    for (const Pfx &p : px) {
        if (p.plen == 32) { k32.push_back({p.a[0]}); v32.push_back({p.value}); }   // /32: hash front
        else b.insert(bswap32(p.a[0]), p.plen, p.value);
        if (image && p.plen > 16 && p.plen < 32) d.longer[bswap32(p.a[0]) >> 16].push_back(p);
    }
    if (b.chunks.empty()) b.chunks.assign(256, 0);
    const size_t nch = b.chunks.size() / 256;
    const size_t cap = image ? nch + std::max<size_t>(nch / 2, 4096) : nch;
    int r = d.l1.upload(b.l1.data(), b.l1.size() * 4);
    if (!r) r = d.chunks.alloc(cap * 1024);
    if (!r && hipMemcpy(d.chunks.p, b.chunks.data(), b.chunks.size() * 4, hipMemcpyHostToDevice) != hipSuccess) r = -EIO;
    // (an image keeps a /32 front with room for as many more, even an empty one)
    const bool front = !k32.empty() || image;
    if (!r && front)
        r = build_hash<Host32Spec>(d.full, k32, v32, 0, nullptr, nullptr, image ? std::max<size_t>(k32.size(), 4096) : 0);
    d.view = r ? Lpm4{nullptr, nullptr, HashTable{}}
               : Lpm4{d.l1.as<uint32_t>(), d.chunks.as<uint32_t>(), front ? d.full.view : HashTable{}};
    d.image = image && !r;
    d.chunk_cap = cap;
    d.chunks_on_dev = nch;
    d.front_live = k32.size();
    if (d.image) { d.hb = std::move(b); d.hb.touched.clear(); }
    else { d.longer.clear(); d.hb = Lpm4Builder{}; d.hb.l1.clear(); d.hb.l1.shrink_to_fit(); }
    return r;
}

// words [lo, hi) of a host image to the same offsets of its device buffer, published
// at the batch boundary (PatchQueue)
int put_words(PatchQueue &pq, const DevBuf &dst, const uint32_t *src, size_t lo, size_t hi)
{
    if (hi <= lo) return 0;
    pq.add(static_cast<uint32_t *>(dst.p) + lo, src + lo, hi - lo);
    return 0;
}

int upload_lpm6(DevLpm6 &d, std::vector<Pfx> &px, size_t room = 0)
{
    std::stable_sort(px.begin(), px.end(), [](const Pfx &x, const Pfx &y) { return x.prio < y.prio; });
    // later (higher priority) entries win for identical (masked addr, plen)
    std::map<std::vector<uint32_t>, uint32_t> uniq;
    std::set<int> lens;
    for (const Pfx &p : px) {
        std::vector<uint32_t> k(5);
        for (int w = 0; w < 4; ++w) {
            int bits = p.plen - 32 * w;
            uint32_t m = bits <= 0 ? 0u : bits >= 32 ? 0xFFFFFFFFu : bswap32(0xFFFFFFFFu << (32 - bits));
            k[w] = p.a[w] & m;
        }
        k[4] = (uint32_t)p.plen;
        uniq[k] = p.value;
        lens.insert(p.plen);
    }
    std::vector<std::vector<uint32_t>> keys, vals;
    d.lens_cnt.clear();
    for (auto &kv : uniq) {
        keys.push_back(kv.first);
        vals.push_back({kv.second});
        d.lens_cnt[(int)kv.first[4]]++;
    }
    int r = build_hash<Lpm6Spec>(d.h, keys, vals, 0, nullptr, nullptr, room ? std::max(keys.size(), room) : 0);
    if (r) return r;
    d.live = keys.size();
    std::vector<uint8_t> l(LENS_CAP, 0);
    std::copy(lens.rbegin(), lens.rend(), l.begin());
    r = d.lens.upload(l.data(), l.size());
    d.view = Lpm6{d.h.view, d.lens.as<uint8_t>(), (uint32_t)lens.size()};
    return r;
}

int compile_cidr_dyn(cv_ctx *c, HostMap *m, bool v6)
{
    if (!m) {
        if (v6) c->cidr6_dyn.view = Lpm6{}; else c->cidr4_dyn.view = Lpm4{nullptr, nullptr, HashTable{}};
        return 0;
    }
    if (!m->is_lpm() || m->ks != (v6 ? 20u : 8u)) return -EINVAL;
    std::vector<Pfx> px;
    m->for_each([&](const uint8_t *k, const uint8_t *) {
        Pfx p{};
        p.prio = rd32(k);
        p.plen = (int)p.prio;
        for (int w = 0; w < (v6 ? 4 : 1); ++w) p.a[w] = rd32(k + 4 + 4 * w);
        p.value = 1;
        px.push_back(p);
    });
    return v6 ? upload_lpm6(c->cidr6_dyn, px) : upload_lpm4(c->cidr4_dyn, px);
}

// cilium_ipcache: a v4 lookup key is {prefixlen 64, pad 0, family 1, ip4, 0...}
// (eps.h:68-86); it matches stored elements with prefixlen <= 64 whose first
// min(prefixlen, 32) bits equal {0, 0, 0, 1}.  Same for v6 with family 2, 160.
int compile_ipcache(cv_ctx *c, HostMap *m)
{
    if (!m) { c->ipc4.view = Lpm4{nullptr, nullptr, HashTable{}}; c->ipc6.view = Lpm6{}; return 0; }
    if (!m->is_lpm() || m->ks != 24 || m->vs < 4) return -EINVAL;
    std::vector<Pfx> p4, p6;
    int err = 0;
    m->for_each([&](const uint8_t *k, const uint8_t *v) {
        const uint32_t plen = rd32(k);
        const uint32_t label = rd32(v);
        for (int fam = 1; fam <= 2; ++fam) {
            const uint8_t want[4] = {0, 0, 0, (uint8_t)fam};
            const uint32_t sbits = plen < 32 ? plen : 32;
            bool match = true;
            for (uint32_t bit = 0; bit < sbits; ++bit) {
                const uint8_t mb = 0x80 >> (bit & 7);
                if ((k[4 + bit / 8] & mb) != (want[bit / 8] & mb)) { match = false; break; }
            }
            if (!match) continue;
            if (fam == 1 && plen > 64) continue;
            if (label & 0x80000000u) { err = -ERANGE; continue; }
            Pfx p{};
            p.prio = plen;
            p.plen = plen > 32 ? (int)(plen - 32) : 0;
            p.value = label;
            for (int w = 0; w < 4; ++w) p.a[w] = rd32(k + 8 + 4 * w);
            (fam == 1 ? p4 : p6).push_back(p);
        }
    });
    if (err) return err;
    int r = upload_lpm4(c->ipc4, p4, true);
    if (!r) r = upload_lpm6(c->ipc6, p6, 4096);
    c->ipc4.of = r ? nullptr : m;
    m->log_clear();
    return r;
}

// The writes logged since the last compile applied in place (the agent's ipcache
// churn: one write used to recompile 100k prefixes, ~32 ms at the batch boundary).
// Each logged key is re-read from the map (present = insert/overwrite, absent =
// delete): a /32 rewrites its bucket of the hash front; a /17-/31 rebuilds the
// subtree of its level-1 slot; a /1-/16 the subtrees of the level-1 slots it spans
// (leaf pushing: a slot's value = the map's longest match for its /16, then the
// longer prefixes inside it in length order, as the full build inserts them).  New
// chunks are appended (the old ones become garbage until the next full build).
// Returns 0 when done, 1 when a full compile is needed, < 0 on error.
// why the last incremental update needed a full compile (CV_REBUILD_WHY prints it)
static const char *rebuild_why = "";
#define NEED_FULL(why)          \
    do {                        \
        rebuild_why = why;      \
        return 1;               \
    } while (0)

int update_ipcache4(cv_ctx *c, HostMap *m)
{
    DevLpm4 &d = c->ipc4;
    if (!m || !d.image || d.of != m || m->log_full) NEED_FULL("no image of this map");
    std::set<uint32_t> dirty;                  // level-1 slots to rebuild
    std::vector<uint64_t> front_b;             // front buckets touched
    HashTable ft{d.full.hb.data(), nullptr, d.full.nb ? d.full.nb - 1 : 0, 0, (uint32_t)Host32Spec::SPB};
    for (const std::vector<uint8_t> &k : m->log) {
        const uint32_t plen = rd32(k.data());
        if (plen < 32) NEED_FULL("a /0 key");               // spans the static bits: both families, /0
        if (k[4] || k[5] || k[6]) continue;    // matches no lookup key
        if (k[7] != 1) continue;               // (IPv6: update_ipcache6)
        if (plen > 64) continue;
        const int len = (int)plen - 32;
        const uint32_t raw = rd32(k.data() + 8), addr = bswap32(raw);
        const uint8_t *v = m->lookup_exact(k.data());
        if (v && (rd32(v) & 0x80000000u)) return -ERANGE;
        if (len == 32) {                       // hash front
            if (!d.full.view.buckets) NEED_FULL("no /32 front");
            if (v) {
                const uint32_t val = rd32(v);
                const int64_t sl = host_find<Host32Spec>(ft, &raw);
                const int64_t s2 = host_upsert<Host32Spec>(ft, &raw, &val);
                if (s2 < 0) NEED_FULL("/32 front probe limit");
                if (sl < 0 && ++d.front_live * 10 > d.full.nb * Host32Spec::SPB * 8) NEED_FULL("/32 front over 80% load");   // > 80 % load
                front_b.push_back((uint64_t)s2 / Host32Spec::SPB);
            } else {
                const int64_t sl = host_find<Host32Spec>(ft, &raw);
                if (sl < 0) continue;
                const uint64_t b = (uint64_t)sl / Host32Spec::SPB;
                uint32_t *w = d.full.hb.data() + b * Host32Spec::BW;
                const int q = (int)(sl % Host32Spec::SPB);
                uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
                tags = (tags & ~(0xFFULL << (8 * q))) | ((uint64_t)TAG_DEAD << (8 * q));
                w[0] = (uint32_t)tags; w[1] = (uint32_t)(tags >> 32);
                front_b.push_back(b);
                --d.front_live;
            }
            continue;
        }
        if (len > 16) {
            const uint32_t x = addr >> 16;
            std::vector<Pfx> &lv = d.longer[x];
            lv.erase(std::remove_if(lv.begin(), lv.end(), [&](const Pfx &p) { return p.prio == plen && p.a[0] == raw; }),
                     lv.end());
            if (v) {
                Pfx p{};
                p.prio = plen; p.plen = len; p.a[0] = raw; p.value = rd32(v);
                lv.push_back(p);
            }
            dirty.insert(x);
        } else {
            const uint32_t span = 1u << (16 - len);
            if (span > 4096) NEED_FULL("a prefix shorter than /4");
            const uint32_t base = (addr >> 16) & ~(span - 1);
            for (uint32_t i = 0; i < span; ++i) dirty.insert(base + i);
        }
    }
    // rebuild the dirty level-1 subtrees on the host image
    uint8_t key[24] = {0};
    key[0] = 48;                               // prefixlen 32 + 16: the longest match of a /16
    key[7] = 1;
    for (const uint32_t x : dirty) {
        const uint32_t raw16 = bswap32(x << 16);
        memcpy(key + 8, &raw16, 4);
        const uint8_t *v0 = m->lookup(key);
        const uint32_t base = v0 ? rd32(v0) : 0u;
        if (base & 0x80000000u) return -ERANGE;
        d.hb.release(d.hb.l1[x]);
        d.hb.l1[x] = base;
        auto it = d.longer.find(x);
        if (it == d.longer.end()) continue;
        if (it->second.empty()) { d.longer.erase(it); continue; }
        std::vector<Pfx> lv = it->second;
        std::stable_sort(lv.begin(), lv.end(), [](const Pfx &a, const Pfx &b) { return a.prio < b.prio; });
        for (const Pfx &p : lv) d.hb.insert(bswap32(p.a[0]), p.plen, p.value);
    }
    const size_t nch = d.hb.chunks.size() / 256;
    if (nch > d.chunk_cap) NEED_FULL("out of device chunk room");           // out of device room: a full build compacts
    PatchQueue &pq = c->pq;
    std::vector<uint32_t> &tc = d.hb.touched;  // new and reused chunks (batches before this
    std::sort(tc.begin(), tc.end());           // publication no longer run: stream order)
    tc.erase(std::unique(tc.begin(), tc.end()), tc.end());
    for (size_t i = 0; i < tc.size();) {
        size_t j = i + 1;
        while (j < tc.size() && tc[j] == tc[j - 1] + 1) ++j;
        put_words(pq, d.chunks, d.hb.chunks.data(), (size_t)tc[i] * 256, ((size_t)tc[j - 1] + 1) * 256);
        i = j;
    }
    tc.clear();
    d.chunks_on_dev = nch;
    for (auto it = dirty.begin(); it != dirty.end();) {          // contiguous runs of slots
        uint32_t lo = *it, hi = lo + 1;
        for (++it; it != dirty.end() && *it == hi; ++it) ++hi;
        put_words(pq, d.l1, d.hb.l1.data(), lo, hi);
    }
    std::sort(front_b.begin(), front_b.end());
    front_b.erase(std::unique(front_b.begin(), front_b.end()), front_b.end());
    for (const uint64_t b : front_b) put_words(pq, d.full.buckets, d.full.hb.data(), b * Host32Spec::BW, (b + 1) * Host32Spec::BW);
    return 0;
}

// The IPv6 ipcache writes logged since the last compile applied in place: a prefix
// is one entry of the per-length hash (Lpm6Spec: the masked address and the length),
// so an insert, overwrite or delete rewrites one bucket; a length that appears or
// disappears rewrites the descending length list the lookup walks.  0 = done, 1 = a
// full compile is needed.
int update_ipcache6(cv_ctx *c, HostMap *m)
{
    DevLpm6 &d = c->ipc6;
    bool any = false;
    for (const std::vector<uint8_t> &k : m->log)
        if (!k[4] && !k[5] && !k[6] && k[7] == 2) { any = true; break; }
    if (!any) return 0;
    if (!d.h.nb || d.h.hb.empty() || !d.lens.p) NEED_FULL("no v6 table");
    HashTable t{d.h.hb.data(), nullptr, d.h.nb - 1, 0, (uint32_t)Lpm6Spec::SPB};
    std::vector<uint64_t> bk;
    bool lens_changed = false;
    for (const std::vector<uint8_t> &k : m->log) {
        const uint32_t plen = rd32(k.data());
        if (plen < 32) NEED_FULL("a /0 key");               // spans the static bits: both families, /0
        if (k[4] || k[5] || k[6] || k[7] != 2 || plen > 160) continue;
        const int len = (int)plen - 32;
        uint32_t key[5];
        for (int w = 0; w < 4; ++w) {
            const int bits = len - 32 * w;
            const uint32_t msk = bits <= 0 ? 0u : bits >= 32 ? 0xFFFFFFFFu : bswap32(0xFFFFFFFFu << (32 - bits));
            key[w] = rd32(k.data() + 8 + 4 * w) & msk;
        }
        key[4] = (uint32_t)len;
        const uint8_t *v = m->lookup_exact(k.data());
        const int64_t old = host_find<Lpm6Spec>(t, key);
        if (v) {
            const uint32_t val = rd32(v);
            if (val & 0x80000000u) return -ERANGE;
            const int64_t sl = host_upsert<Lpm6Spec>(t, key, &val);
            if (sl < 0) NEED_FULL("v6 probe limit");
            if (old < 0) {
                if (++d.live * 10 > d.h.nb * Lpm6Spec::SPB * 8) NEED_FULL("v6 table over 80% load");   // > 80 % load
                if (d.lens_cnt[len]++ == 0) lens_changed = true;
            }
            bk.push_back((uint64_t)sl / Lpm6Spec::SPB);
        } else if (old >= 0) {
            const uint64_t b = (uint64_t)old / Lpm6Spec::SPB;
            uint32_t *w = d.h.hb.data() + b * Lpm6Spec::BW;
            const int q = (int)(old % Lpm6Spec::SPB);
            uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
            tags = (tags & ~(0xFFULL << (8 * q))) | ((uint64_t)TAG_DEAD << (8 * q));
            w[0] = (uint32_t)tags; w[1] = (uint32_t)(tags >> 32);
            bk.push_back(b);
            --d.live;
            if (--d.lens_cnt[len] == 0) { d.lens_cnt.erase(len); lens_changed = true; }
        }
    }
    std::sort(bk.begin(), bk.end());
    bk.erase(std::unique(bk.begin(), bk.end()), bk.end());
    for (const uint64_t b : bk) put_words(c->pq, d.h.buckets, d.h.hb.data(), b * Lpm6Spec::BW, (b + 1) * Lpm6Spec::BW);
    if (lens_changed) {
        uint32_t lw[LENS_CAP / 4] = {0};
        uint8_t *l = reinterpret_cast<uint8_t *>(lw);
        size_t n = 0;
        for (auto it = d.lens_cnt.rbegin(); it != d.lens_cnt.rend(); ++it) l[n++] = (uint8_t)it->first;
        c->pq.add(d.lens.p, lw, LENS_CAP / 4);
        d.view.nlens = (uint32_t)n;
    }
    return 0;
}

// both families' incremental ipcache writes, or 1 (a full compile; nothing published)
int update_ipcache(cv_ctx *c, HostMap *m)
{
    const size_t mk = c->pq.mark();
    int r = update_ipcache4(c, m);
    if (!r) r = update_ipcache6(c, m);
    if (r) c->pq.undo(mk);
    else m->log_clear();
    return r;
}

// policy map -> PolicySpec table (proxy_port inline, so a lookup is one line) + 32-B
// side values {proxy_port, pad, packets, bytes}; device counters of entries the
// agent did not rewrite since the last sync are carried over.
int compile_policy(cv_ctx *c, MapObj *mo)
{
    (void)c;
    HostMap *m = mo->hm.get();
    if (m->ks != 8 || m->vs != 24 || m->is_lpm()) return -EINVAL;
    if (mo->pol.view.buckets) {
        std::vector<uint8_t> dv(mo->pol.vals.n);
        if (hipMemcpy(dv.data(), mo->pol.vals.p, dv.size(), hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
        HashTable old{mo->pol.hb.data(), nullptr, mo->pol.nb - 1, 32, PolicySpec::SPB};
        m->for_each([&](const uint8_t *k, const uint8_t *v) {
            if (mo->written.count(kstr(k, 8))) return;
            uint32_t kw[2] = {rd32(k), rd32(k + 4)};
            int64_t s = host_find<PolicySpec>(old, kw);
            if (s >= 0) memcpy(const_cast<uint8_t *>(v) + 8, &dv[(size_t)s * 32 + 8], 16);
        });
    }
    mo->written.clear();
    std::vector<std::vector<uint32_t>> keys, proxy;
    std::vector<uint8_t> vals;
    m->for_each([&](const uint8_t *k, const uint8_t *v) {
        keys.push_back({rd32(k), rd32(k + 4)});
        proxy.push_back({(uint32_t)v[0] | (uint32_t)v[1] << 8});   // raw be16 bytes, as stored
        size_t o = vals.size();
        vals.resize(o + 32, 0);
        memcpy(&vals[o], v, 24);
    });
    std::vector<int64_t> slots;
    int r = build_hash<PolicySpec>(mo->pol, keys, proxy, 32, &vals, &slots);
    if (r) return r;
    // counter deltas: one 64-bit word per slot, apart from the value lines so the
    // datapath's atomics do not share lines with proxy_port reads
    const size_t nslots = mo->pol.nb * PolicySpec::SPB;
    if ((r = mo->pol.aux.alloc(nslots * 8))) return r;
    if (hipMemset(mo->pol.aux.p, 0, nslots * 8) != hipSuccess) return -EIO;
    mo->pol.view.aux = mo->pol.aux.as<unsigned long long>();
    mo->pol_version = m->version;
    mo->pol_live = keys.size();
    m->log_clear();
    return 0;
}

// The policy writes logged since the last compile applied in place: a written key's
// bucket (its inline proxy_port) and 32-B side value {proxy_port, pad, packets, bytes}
// take the agent's value, its counter-delta word is cleared; a deleted key's slot
// becomes a tombstone.  Every other entry keeps its device-resident counters, as the
// full compile carries them over.  0 = done, 1 = a full compile is needed.
int update_policy(cv_ctx *c, MapObj *mo)
{
    HostMap *m = mo->hm.get();
    DevHash &d = mo->pol;
    if (!d.view.buckets || m->log_full || d.hb.empty()) return 1;
    HashTable t{d.hb.data(), nullptr, d.nb - 1, 32, (uint32_t)PolicySpec::SPB};
    std::vector<uint64_t> bk;
    struct Side { int64_t s; uint8_t v[32]; };
    std::vector<Side> side;
    for (const std::vector<uint8_t> &k : m->log) {
        const uint32_t kw[2] = {rd32(k.data()), rd32(k.data() + 4)};
        const uint8_t *v = m->lookup_exact(k.data());
        const int64_t old = host_find<PolicySpec>(t, kw);
        if (v) {
            const uint32_t px = (uint32_t)v[0] | (uint32_t)v[1] << 8;   // raw be16 bytes, as stored
            const int64_t sl = host_upsert<PolicySpec>(t, kw, &px);
            if (sl < 0) return 1;
            if (old < 0 && ++mo->pol_live * 10 > d.nb * PolicySpec::SPB * 8) return 1;   // > 80 % load
            Side e{sl, {0}};
            memcpy(e.v, v, 24);
            side.push_back(e);
            bk.push_back((uint64_t)sl / PolicySpec::SPB);
        } else if (old >= 0) {
            const uint64_t b = (uint64_t)old / PolicySpec::SPB;
            uint32_t *w = d.hb.data() + b * PolicySpec::BW;
            const int q = (int)(old % PolicySpec::SPB);
            uint64_t tags = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
            tags = (tags & ~(0xFFULL << (8 * q))) | ((uint64_t)TAG_DEAD << (8 * q));
            w[0] = (uint32_t)tags; w[1] = (uint32_t)(tags >> 32);
            bk.push_back(b);
            --mo->pol_live;
        }
    }
    std::sort(bk.begin(), bk.end());
    bk.erase(std::unique(bk.begin(), bk.end()), bk.end());
    for (const uint64_t b : bk) put_words(c->pq, d.buckets, d.hb.data(), b * PolicySpec::BW, (b + 1) * PolicySpec::BW);
    const uint32_t zero[2] = {0, 0};
    for (const Side &e : side) {          // in log order: the last write of a key wins
        c->pq.add(d.vals.as<uint8_t>() + (size_t)e.s * 32, e.v, 8);
        c->pq.add(d.aux.as<unsigned long long>() + e.s, zero, 2);
    }
    mo->written.clear();
    mo->pol_version = m->version;
    m->log_clear();
    return 0;
}

// CT table sized for max_entries at 60 % bucket load, filled on the device from the
// agent's entries (k_ct_load); v6 tables hold struct ipv6_ct_tuple keys (40 B) in
// Ct6Spec buckets.  From here on the device copy is authoritative: the host store is
// emptied and every map operation goes to HBM.
template <class S>
int compile_ct_t(cv_ctx *c, MapObj *mo, uint32_t ks, int kind)
{
    HostMap *m = mo->hm.get();
    if (m->ks != ks || m->vs != 56) return -EINVAL;
    const uint64_t n = m->count();
    DevHash &d = mo->ct;
    const uint64_t nb = buckets_for(std::max<uint64_t>(m->max_entries, n), S::SPB);
    int r = d.buckets.alloc(nb * S::BW * 4);
    if (!r) r = d.vals.alloc(nb * S::SPB * CT_COLD);          // side slots (the hot words sit in the buckets)
    if (!r) r = mo->live.alloc(8);
    if (r) return r;
    if (hipMemset(d.buckets.p, 0, d.buckets.n) != hipSuccess || hipMemset(d.vals.p, 0, d.vals.n) != hipSuccess)
        return -EIO;
    d.nb = nb;
    d.view = HashTable{d.buckets.as<uint32_t>(), d.vals.as<uint8_t>(), nb - 1, CT_COLD, (uint32_t)S::SPB, nullptr,
                       mo->live.as<unsigned long long>(), m->max_entries};
    if (n) {
        std::vector<uint32_t> kw((size_t)n * S::KW, 0), vw((size_t)n * 16, 0);
        size_t i = 0;
        m->for_each([&](const uint8_t *k, const uint8_t *v) {
            memcpy(&kw[i * S::KW], k, ks);
            memcpy(&vw[i * 16], v, 56);
            ++i;
        });
        DevBuf dk, dv, df;
        if ((r = dk.upload(kw.data(), kw.size() * 4)) || (r = dv.upload(vw.data(), vw.size() * 4)) || (r = df.alloc(4)))
            return r;
        uint32_t fail = 0;
        if (hipMemset(df.p, 0, 4) != hipSuccess) return -EIO;
        if (launch_ct_load(d.view, kind == MK_CT6, dk.as<uint32_t>(), dv.as<uint32_t>(), n, df.as<uint32_t>(), nullptr))
            return -EIO;
        if (hipMemcpy(&fail, df.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
        if (fail) return -E2BIG;
    }
    if (hipMemcpy(mo->live.p, &n, 8, hipMemcpyHostToDevice) != hipSuccess) return -EIO;
    mo->live_upper = n;
    mo->cap = m->max_entries;
    m->clear();
    mo->kind = kind;
    mo->ct_id = c->next_ct_id++;
    mo->gen++;
    return 0;
}

int compile_ct(cv_ctx *c, MapObj *mo) { return compile_ct_t<Ct4Spec>(c, mo, 14, MK_CT4); }
int compile_ct6(cv_ctx *c, MapObj *mo) { return compile_ct_t<Ct6Spec>(c, mo, 40, MK_CT6); }

// cilium_lb{4,6}_services: lb{4,6}_key -> lb{4,6}_service, values inline
int compile_lb(cv_ctx *c, HostMap *m, bool v6)
{
    DevHash &d = v6 ? c->lb6 : c->lb4;
    if (!m) { d.view = HashTable{}; return 0; }
    const uint32_t ks = v6 ? 20 : 8, vs = v6 ? 24 : 12;
    if (m->is_lpm() || m->ks != ks || m->vs != vs) return -EINVAL;
    std::vector<std::vector<uint32_t>> keys, vals;
    m->for_each([&](const uint8_t *k, const uint8_t *v) {
        std::vector<uint32_t> kw(ks / 4), vw(vs / 4);
        memcpy(kw.data(), k, ks);
        memcpy(vw.data(), v, vs);
        keys.push_back(kw);
        vals.push_back(vw);
    });
    return v6 ? build_hash<Lb6Spec>(d, keys, vals, 0, nullptr, nullptr)
              : build_hash<Lb4Spec>(d, keys, vals, 0, nullptr, nullptr);
}

// cilium_lb{4,6}_reverse_nat: u16 key -> dense table [65536] {address, port | valid << 16}
int compile_revnat(cv_ctx *c, HostMap *m, bool v6)
{
    DevBuf &d = v6 ? c->revnat6 : c->revnat4;
    if (!m) { d.release(); return 0; }
    const uint32_t vs = v6 ? 18 : 6, w = v6 ? 8 : 2;
    if (m->is_lpm() || m->ks != 2 || m->vs != vs) return -EINVAL;
    std::vector<uint32_t> tab((size_t)65536 * w, 0);
    m->for_each([&](const uint8_t *k, const uint8_t *v) {
        const uint32_t idx = rd16(k);
        uint32_t *e = &tab[(size_t)idx * w];
        const uint32_t na = v6 ? 4 : 1;
        memcpy(e, v, na * 4);
        e[na] = rd16(v + na * 4) | (1u << 16);
    });
    return d.upload(tab.data(), tab.size() * 4);
}

void drain(cv_ctx *c);

// The stream of the batch about to be submitted waits (on the device) for the last
// batch or publication of this context, whatever stream that was on: a context's
// batches and table publications are totally ordered, so a publication never races a
// batch of another stream and the per-launch group scratch is never shared by two
// batches in flight.  No host wait.
void order_stream(cv_ctx *c, hipStream_t s)
{
    if (c->have_last && c->last_stream != s) (void)hipStreamWaitEvent(s, c->last_ev, 0);
}

void mark_stream(cv_ctx *c, hipStream_t s)
{
    if (!c->last_ev && hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming) != hipSuccess) return;
    (void)hipEventRecord(c->last_ev, s);
    c->last_stream = s;
    c->have_last = true;
}

// order_stream now, mark_stream on every exit (error returns included: kernels of a
// partly submitted launch are still queued on s, and the next publication or batch on
// another stream must wait for them)
struct StreamScope {
    cv_ctx *c;
    hipStream_t s;
    StreamScope(cv_ctx *cc, hipStream_t ss) : c(cc), s(ss) { order_stream(c, s); }
    ~StreamScope() { mark_stream(c, s); }
};

// The queued table patches to the device, in stream s: pinned staging (a buffer whose
// previous publication has completed, else a new one), one async copy, k_patch.
int publish(cv_ctx *c, hipStream_t s)
{
    PatchQueue &pq = c->pq;
    if (pq.recs.empty()) return 0;
    const size_t rb = pq.recs.size() * sizeof(PatchRec), bytes = rb + pq.words.size() * 4;
    Staging *st = nullptr;
    for (Staging &x : c->staging) {
        if (x.cap < bytes) continue;
        if (x.done && hipEventQuery(x.done) != hipSuccess) {
            (void)hipGetLastError();              // (hipErrorNotReady is sticky: the next launch check would see it)
            continue;
        }
        st = &x;
        break;
    }
    if (!st) {
        Staging x;
        x.cap = std::max<size_t>(bytes, 1 << 16);
        if (hipHostMalloc(&x.host, x.cap, hipHostMallocDefault) != hipSuccess) return -ENOMEM;
        if (hipMalloc(&x.dev, x.cap) != hipSuccess) { (void)hipHostFree(x.host); return -ENOMEM; }
        if (hipEventCreateWithFlags(&x.done, hipEventDisableTiming) != hipSuccess) return -ENOMEM;
        c->staging.push_back(x);
        st = &c->staging.back();
    }
    memcpy(st->host, pq.recs.data(), rb);
    memcpy(static_cast<uint8_t *>(st->host) + rb, pq.words.data(), pq.words.size() * 4);
    order_stream(c, s);
    if (hipMemcpyAsync(st->dev, st->host, bytes, hipMemcpyHostToDevice, s) != hipSuccess) return -EIO;
    const int r = launch_patches(static_cast<const PatchRec *>(st->dev), (uint32_t)pq.recs.size(),
                                 reinterpret_cast<const uint32_t *>(static_cast<uint8_t *>(st->dev) + rb), s);
    if (r) return r;
    (void)hipEventRecord(st->done, s);
    mark_stream(c, s);
    pq.recs.clear();
    pq.words.clear();
    ++c->publications;
    return 0;
}

// Queued patches hold raw addresses of the device buffers live now.  They go out before
// any buffer is replaced (a rebuild) and on every error exit of a boundary, so no patch
// outlives the buffer it targets (a later sync could free and reallocate it).  A
// publication that fails drops the queue and makes the next boundary compile the
// incremental tables in full, so the host images and the device agree again.
int flush_patches(cv_ctx *c, hipStream_t s)
{
    if (c->pq.recs.empty()) return 0;
    const int r = publish(c, s);
    if (r) {
        c->pq.recs.clear();
        c->pq.words.clear();
        c->force_full = true;
    }
    return r;
}

// the test hook CV_INJECT_COMPILE_FAIL=<role>: that role's next full compile fails
bool injected_failure(int role)
{
    const char *e = getenv("CV_INJECT_COMPILE_FAIL");
    return e && atoi(e) == role;
}

int sync_body(cv_ctx *c, hipStream_t stream);

// Apply the agent's writes since the last batch boundary to the device tables, for a
// batch about to run on stream s.  Incremental writes (ipcache v4 and v6 prefixes,
// policy entries) are published in stream order (PatchQueue): no device wait.  A
// table that has to be rebuilt (other roles, endpoint changes, a write the incremental
// path cannot apply) replaces device buffers: only then does the boundary wait for
// the batches already submitted.  All or nothing per table: a table whose compile fails
// keeps its old version (the next boundary retries it), and the patches already queued
// for other tables are published against the buffers they were made for.
// a kernel of an earlier batch met a list word past its launch (GroupScratch::err): the
// device state of that batch is unknown, every later call fails
int walker_error(cv_ctx *c)
{
    if (c->gerr_host && __atomic_load_n(c->gerr_host, __ATOMIC_ACQUIRE)) {
        fprintf(stderr, "[cv] a conntrack stage read a list word past its launch (error %#x)\n", *c->gerr_host);
        return -EPROTO;
    }
    return 0;
}

int sync_locked(cv_ctx *c, hipStream_t stream = nullptr)
{
    if (const int e = walker_error(c)) return e;
    const int r = sync_body(c, stream);
    if (r) (void)flush_patches(c, stream);
    return r;
}

int sync_body(cv_ctx *c, hipStream_t stream)
{
    if (c->force_full) {                       // a lost publication: recompile the incremental tables
        c->role_version[CV_ROLE_IPCACHE] = ~0ull;
        for (auto &e : c->eps)
            if (MapObj *p = get(c, e.policy)) p->pol_version = ~0ull;
    }
    bool dirty = c->eps_dirty;
    for (int r = 0; r < CV_NUM_ROLES; ++r) {
        MapObj *m = get(c, c->role[r]);
        uint64_t v = m ? m->hm->version : 0;
        if (v != c->role_version[r]) dirty = true;
    }
    for (auto &e : c->eps) {
        MapObj *p = get(c, e.policy);
        if (p && p->hm->version != p->pol_version) dirty = true;
    }
    if (!dirty) return 0;
    int r = set_device(c);
    if (r) return r;
    bool drained = false;
    auto rebuild = [&]() {                     // no batch may still read a table we replace
        int e = flush_patches(c, stream);      // (queued patches target the buffers live now)
        if (!drained) { drain(c); drained = true; }
        ++c->full_compiles;
        return e;
    };
    const bool full = c->force_full || getenv("CV_NO_INCREMENTAL");
    for (int role = 0; role < CV_NUM_ROLES; ++role) {
        MapObj *m = get(c, c->role[role]);
        uint64_t v = m ? m->hm->version : 0;
        if (v == c->role_version[role]) continue;
        HostMap *hm = m ? m->hm.get() : nullptr;
        if (role == CV_ROLE_IPCACHE) {
            r = full ? 1 : update_ipcache(c, hm);
            if (r == 1 && getenv("CV_REBUILD_WHY")) fprintf(stderr, "[cv] ipcache rebuild: %s\n", rebuild_why);
            if (r == 1 && !(r = rebuild())) r = injected_failure(role) ? -EIO : compile_ipcache(c, hm);
        } else {
            if ((r = rebuild())) return r;
            if (injected_failure(role)) return -EIO;
            switch (role) {
            case CV_ROLE_CIDR4_FIX: r = compile_cidr_fix(c, hm, false); break;
            case CV_ROLE_CIDR6_FIX: r = compile_cidr_fix(c, hm, true); break;
            case CV_ROLE_CIDR4_DYN: r = compile_cidr_dyn(c, hm, false); break;
            case CV_ROLE_CIDR6_DYN: r = compile_cidr_dyn(c, hm, true); break;
            case CV_ROLE_LXC: r = compile_lxc(c, hm); break;
            case CV_ROLE_LB4_SERVICES: r = compile_lb(c, hm, false); break;
            case CV_ROLE_LB6_SERVICES: r = compile_lb(c, hm, true); break;
            case CV_ROLE_LB4_REVNAT: r = compile_revnat(c, hm, false); break;
            case CV_ROLE_LB6_REVNAT: r = compile_revnat(c, hm, true); break;
            default: r = 0; break;
            }
        }
        if (r) return r;
        c->role_version[role] = v;
    }
    bool eps_changed = c->eps_dirty;
    for (auto &e : c->eps) {
        MapObj *p = get(c, e.policy);
        if (p && p->hm->version != p->pol_version) {
            const size_t mk = c->pq.mark();
            r = full ? 1 : update_policy(c, p);
            if (r == 1) {
                c->pq.undo(mk);
                if ((r = rebuild())) return r;
                r = compile_policy(c, p);
                eps_changed = true;
            }
            if (r) return r;
        }
    }
    if (eps_changed) {
        if ((r = rebuild())) return r;
        if (injected_failure(CV_NUM_ROLES)) return -EIO;    // (the endpoint table)
        std::vector<EpDev> ev;
        std::vector<EpHot> hot, hot6;
        std::vector<uint16_t> of(65536, 0);
        for (size_t i = 0; i < c->eps.size(); ++i) {
            const Endpoint &e = c->eps[i];
            EpDev d{};
            MapObj *p = get(c, e.policy);
            MapObj *t = get(c, e.ct4);
            MapObj *t6 = get(c, e.ct6);
            if (p) d.policy = p->pol.view;
            if (t) { d.ct4 = t->ct.view; d.ct_id = t->ct_id; }
            if (t6) d.ct6 = t6->ct.view;
            d.seclabel = e.seclabel;
            d.lxc_id = e.lxc_id;
            d.ipv4 = e.ipv4;
            for (int j = 0; j < 4; ++j) d.ipv6[j] = e.ipv6[j];
            for (int j = 0; j < 2; ++j) { d.mac[j] = e.mac[j]; d.node_mac[j] = e.node_mac[j]; }
            ev.push_back(d);
            const uint32_t v4 = (d.ct_id & EPH_CT_ID) | (d.ipv4 ? EPH_V4 : 0u);
            EpHot h{d.policy.buckets, d.policy.vals, d.policy.aux, d.ct4.buckets, d.ct4.vals, d.ct4.live,
                    (uint32_t)d.policy.mask, (uint32_t)d.ct4.mask, d.seclabel, v4};
            EpHot h6{d.policy.buckets, d.policy.vals, d.policy.aux, d.ct6.buckets, d.ct6.vals, d.ct6.live,
                     (uint32_t)d.policy.mask, (uint32_t)d.ct6.mask, d.seclabel, v4};
            if ((d.policy.buckets && d.policy.vstride != 32) || (d.ct4.buckets && d.ct4.vstride != CT_COLD) ||
                (d.ct6.buckets && d.ct6.vstride != CT_COLD) || d.policy.mask > 0xFFFFFFFFull ||
                d.ct4.mask > 0xFFFFFFFFull || d.ct6.mask > 0xFFFFFFFFull)
                return -EINVAL;                                   // (EpHot's fixed strides and 32-bit masks)
            hot.push_back(h);
            hot6.push_back(h6);
            of[e.lxc_id] = (uint16_t)(i + 1);
        }
        // one policy and CT4 map for every endpoint, each with LXC_IPV4: the netdev stages'
        // common line (DpParams::uni4)
        c->uni4_on = !hot.empty();
        for (size_t i = 0; i < hot.size() && c->uni4_on; ++i)
            c->uni4_on = hot[i].pol_buckets == hot[0].pol_buckets && hot[i].ct_buckets == hot[0].ct_buckets &&
                         hot[i].ct_v4 == hot[0].ct_v4 && (hot[i].ct_v4 & EPH_V4);
        if (c->uni4_on) c->uni4 = hot[0];
        c->uni6_on = !hot6.empty();
        for (size_t i = 0; i < hot6.size() && c->uni6_on; ++i)
            c->uni6_on = hot6[i].pol_buckets == hot6[0].pol_buckets && hot6[i].ct_buckets == hot6[0].ct_buckets;
        if (c->uni6_on) c->uni6 = hot6[0];
        if (ev.empty()) { ev.push_back(EpDev{}); hot.push_back(EpHot{}); hot6.push_back(EpHot{}); }
        r = c->eps_dev.upload(ev.data(), ev.size() * sizeof(EpDev));
        if (!r) r = c->ephot_dev.upload(hot.data(), hot.size() * sizeof(EpHot));
        if (!r) r = c->ephot6_dev.upload(hot6.data(), hot6.size() * sizeof(EpHot));
        if (!r) r = c->ep_of_lxc.upload(of.data(), of.size() * 2);
        if (r) return r;
        c->eps_dirty = false;
    }
    c->force_full = false;
    return flush_patches(c, stream);
}

DpParams params(cv_ctx *c)
{
    DpParams p{};
    p.flags = c->flags;
    if (c->hk.coarse_groups) p.flags |= F_TEST_COARSE_GROUPS;
    p.win_lo = 0;
    p.win_span = ~0u;
    p.n_eps = (uint32_t)c->eps.size();
    p.cidr4_fix = c->role[CV_ROLE_CIDR4_FIX] >= 0 ? c->cidr4_fix.view : HashTable{};
    p.cidr6_fix = c->role[CV_ROLE_CIDR6_FIX] >= 0 ? c->cidr6_fix.view : HashTable{};
    p.lxc4 = c->role[CV_ROLE_LXC] >= 0 ? c->lxc4.view : HashTable{};
    p.lxc6 = c->role[CV_ROLE_LXC] >= 0 ? c->lxc6.view : HashTable{};
    p.cidr4_dyn = c->role[CV_ROLE_CIDR4_DYN] >= 0 ? c->cidr4_dyn.view : Lpm4{nullptr, nullptr, HashTable{}};
    p.cidr6_dyn = c->role[CV_ROLE_CIDR6_DYN] >= 0 ? c->cidr6_dyn.view : Lpm6{};
    p.ipc4 = c->role[CV_ROLE_IPCACHE] >= 0 ? c->ipc4.view : Lpm4{nullptr, nullptr, HashTable{}};
    p.ipc6 = c->role[CV_ROLE_IPCACHE] >= 0 ? c->ipc6.view : Lpm6{};
    p.eps = c->eps_dev.as<EpDev>();
    p.ephot = c->ephot_dev.as<EpHot>();
    p.ephot6 = c->ephot6_dev.as<EpHot>();
    p.uni4_on = c->uni4_on && !c->hk.no_uni ? 1u : 0u;
    p.uni4 = c->uni4;
    p.uni6_on = c->uni6_on && !c->hk.no_uni ? 1u : 0u;
    p.uni6 = c->uni6;
    p.ep_of_lxc = c->ep_of_lxc.as<uint16_t>();
    p.metrics = c->metrics;
    p.lb4 = c->role[CV_ROLE_LB4_SERVICES] >= 0 ? c->lb4.view : HashTable{};
    p.lb6 = c->role[CV_ROLE_LB6_SERVICES] >= 0 ? c->lb6.view : HashTable{};
    p.revnat4 = c->role[CV_ROLE_LB4_REVNAT] >= 0 ? c->revnat4.as<uint32_t>() : nullptr;
    p.revnat6 = c->role[CV_ROLE_LB6_REVNAT] >= 0 ? c->revnat6.as<uint32_t>() : nullptr;
    p.v4_cluster_mask = c->node.ipv4_cluster_mask;
    p.v4_cluster_range = c->node.ipv4_cluster_range;
    p.v4_loopback = c->node.ipv4_loopback;
    memcpy(p.router6, c->node.router_ip6, 16);
    p.host_mac[0] = p.host_mac[1] = 0;
    memcpy(p.host_mac, c->node.host_mac, 6);
    p.net_mac[0] = p.net_mac[1] = 0;
    memcpy(p.net_mac, c->node.net_mac, 6);
    p.notify = reinterpret_cast<uint32_t *>(c->notify);
    p.notify_cap = c->notify_cap;
    p.notify_count = c->notify_count;
    p.trace = reinterpret_cast<uint32_t *>(c->trace);
    p.trace_cap = c->trace_cap;
    p.trace_count = c->trace_count;
    p.trace_agg = c->trace_agg;
    p.ingress_ifindex = c->ingress_ifindex;
    return p;
}

int check_batch(const cv_batch *b)
{
    if (!b || (!b->frames && b->n) || (!b->len && b->n)) return -EINVAL;
    if (b->stride < 64 || (b->stride & 15)) return -EINVAL;
    if ((reinterpret_cast<uintptr_t>(b->frames) & 15)) return -EINVAL;
    return 0;
}

BatchDev to_dev(const cv_batch *b) { return BatchDev{b->frames, b->stride, b->n, b->len, b->mark, 0, nullptr}; }

// packets [off, off + n) of a batch / its outputs
BatchDev chunk(const cv_batch *b, uint32_t off, uint32_t n)
{
    return BatchDev{b->frames + (size_t)off * b->stride, b->stride, n, b->len + off, b->mark ? b->mark + off : nullptr,
                    off, nullptr};
}

OutDev to_dev(const cv_out *o)
{
    OutDev d{};
    if (o) {
        d.xdp = o->xdp; d.ret = o->ret; d.identity = o->identity; d.ct = o->ct; d.proxy = o->proxy;
        d.nl = o->nl; d.nu = o->nu; d.reason = o->reason; d.frames = o->frames_out;
    }
    return d;
}

OutDev chunk(const cv_out *o, uint32_t off, uint32_t stride = 0)
{
    OutDev d = to_dev(o);
    if (d.frames) d.frames += (size_t)off * stride;
    if (d.xdp) d.xdp += off;
    if (d.ret) d.ret += off;
    if (d.identity) d.identity += off;
    if (d.ct) d.ct += off;
    if (d.proxy) d.proxy += off;
    if (d.nl) d.nl += off;
    if (d.nu) d.nu += off;
    if (d.reason) d.reason += off;
    return d;
}

// per-launch group scratch: a node table of >= 2 (ingress) / 8 (egress: up to five
// address-pair nodes per packet) slots per packet, so probing always terminates
int ensure_groups(cv_ctx *c, uint32_t cmax, bool egress)
{
    const uint64_t per = egress ? 8 : 2;
    if (cmax <= c->gn && (!egress || c->g_egress) && c->gcap >= per * cmax) return 0;
    cmax = std::max<uint32_t>(cmax, (uint32_t)c->gn);
    uint64_t cap = 1024;
    while (cap < per * cmax || cap < c->gcap) cap <<= 1;
    (void)hipDeviceSynchronize();
    if (c->gtable.alloc(cap * 16) || c->gsingle.alloc((size_t)cmax * 4) ||
        c->gpkey.alloc((size_t)cmax * 8) || c->gent.alloc((size_t)cmax * 8) || c->gbig.alloc((size_t)cmax * 16) ||
        c->gsjob.alloc(((size_t)cmax / 4096 + 16) * SJOB_WORDS * 4) ||
        c->gbx.alloc(((size_t)GBIN_MAX + ((size_t)cmax / BIG_MIN + 2) * BIGW) * 4) ||
        c->ghot.alloc(((size_t)(cmax / 1024 + 256) * 24 + 4096) * 4) ||
        c->gcnt.alloc(((size_t)GBIN_MAX * GBLK + 1 + 1024) * 4) || c->gwork6.alloc((size_t)cmax * 4) ||
        c->ghword.alloc((size_t)cmax * 4) ||
        c->ghcnt.alloc(((size_t)32 * (cmax / 4096 + 1) + 1 + 1024) * 4) ||
        c->gslot.alloc((size_t)cmax * 4) || c->gnext.alloc((size_t)cmax * 4) ||
        c->gsrec.alloc((size_t)cmax * 32) ||
        c->gorder.alloc((size_t)cmax * 8) || c->gwork.alloc((size_t)cmax * 4) || c->gifx.alloc((size_t)cmax * 4) ||
        c->gcursor.alloc(CURSOR_WORDS * 4) ||
        c->gqueue.alloc(((size_t)cmax / QSPLIT + 512) * QSPLIT * QBANKS * 4))
        return -ENOMEM;
    (void)hipMemset(c->gtable.p, 0, cap * 16);
    if (egress || c->g_egress) {
        if (c->gparent.alloc(cap * 8) || c->geg.alloc((size_t)cmax * EG_WORDS * 4) ||
            c->gdel.alloc((size_t)cmax * DEL_SLOTS * 16) || c->gest.alloc((size_t)cmax * 64) ||
            c->gres.alloc((size_t)cmax * 16) || c->gdel_ev.alloc((size_t)cmax * 32))
            return -ENOMEM;
        (void)hipMemset(c->gparent.p, 0, cap * 8);
        c->g_egress = true;
    }
    c->gcap = cap;
    c->gn = cmax;
    c->epoch = 0;
    return 0;
}

// log2 of the bins of a binned grouping of n packets: bins of about 2^GBIN_LOG entries
// (CV_GBIN_LOG overrides, for measurements), at most GBIN_MAX bins
uint32_t gbin_bits(uint32_t n)
{
    static const int lg = [] {
        const char *e = getenv("CV_GBIN_LOG");
        const int v = e ? atoi(e) : 10;
        return v >= 8 && v <= 12 ? v : 10;
    }();
    uint32_t b = 4;
    while (b < 14 && (1ull << (b + lg)) < n) ++b;
    return b;
}

// the scratch view for the next launch, which uses `epochs` fresh epochs
GroupScratch next_groups(cv_ctx *c, uint32_t epochs, hipStream_t stream)
{
    if (c->epoch + epochs < c->epoch || c->epoch == 0) {   // start, or 2^32 launches: clear stale tags
        (void)hipMemsetAsync(c->gtable.p, 0, c->gcap * 16, stream);
        if (c->gparent.p) (void)hipMemsetAsync(c->gparent.p, 0, c->gcap * 8, stream);
        c->epoch = 0;
    }
    GroupScratch gs{c->gtable.as<unsigned long long>(), (uint32_t)(c->gcap - 1), c->epoch + 1,
                    c->gslot.as<uint32_t>(), c->gnext.as<uint32_t>(), c->gsrec.as<uint4>(),
                    c->gparent.as<unsigned long long>(), c->geg.as<uint32_t>(),
                    ++c->serial, c->gorder.as<uint32_t>(), c->gcursor.as<uint32_t>(), c->gqueue.as<uint32_t>(),
                    (uint32_t)(c->gn / QSPLIT + 512), c->gwork.as<uint32_t>(), c->gifx.as<uint32_t>(),
                    c->gsingle.as<uint32_t>(), c->gpkey.as<unsigned long long>(), c->gent.as<uint2>(),
                    c->gcnt.as<uint32_t>(), c->gbig.as<unsigned long long>(), 4, c->gnext.as<uint32_t>(),
                    c->gwork6.as<uint32_t>(), c->ghword.as<uint32_t>(), c->ghcnt.as<uint32_t>(), (uint32_t)Q_NETDEV,
                    0};
    gs.del = c->gdel.as<uint4>();
    gs.res = c->gres.as<uint4>();
    gs.del_ev = c->gdel_ev.as<uint4>();
    gs.est = c->gest.as<uint4>();
    gs.q6 = (uint32_t)Q_NETDEV6;
    gs.err = c->gerr_dev;
    gs.sjob = c->gsjob.as<uint32_t>();
    gs.sjob_cap = (uint32_t)(c->gn / 4096 + 16);
    gs.hot = c->ghot.as<uint32_t>();
    gs.hot_chunks = (uint32_t)(c->gn / 1024 + 256);
    gs.gbx = c->gbx.as<uint32_t>();
    gs.gbx_cap = (uint32_t)(c->gn / BIG_MIN + 2);
    (void)hipMemsetAsync(c->gcursor.p, 0, CURSOR_WORDS * 4, stream);
    c->epoch += epochs;
    return gs;
}

// diagnostics (CV_GROUP_STATS): per node-table queue (services, NAT writers) groups per
// size class; per binned conntrack queue (flat: egress components, else netdev runs)
// runs by size (powers of two), packets in runs past 64, the largest run
void group_stats(cv_ctx *c, const char *what, hipStream_t stream, bool flat)
{
    std::vector<uint32_t> cur(CURSOR_WORDS);
    (void)hipStreamSynchronize(stream);
    (void)hipMemcpy(cur.data(), c->gcursor.p, CURSOR_WORDS * 4, hipMemcpyDeviceToHost);
    static const char *qn[NQUEUES] = {"netdev", "lb4", "lb6", "ct4", "ct6", "nat"};
    for (int q : {(int)Q_LB4, (int)Q_LB6, (int)Q_NAT}) {
        uint64_t groups = 0;
        for (int k = 0; k < QSPLIT; ++k) groups += cur[qctr(q, k)];
        if (!groups) continue;
        fprintf(stderr, "[cv groups] %s %s: %llu groups, largest %u; by class:", what, qn[q],
                (unsigned long long)groups, cur[GMAX_WORD0 + q]);
        for (int k = 0; k < NCLASS; ++k) fprintf(stderr, " %u", cur[qcls(q, k)]);
        fprintf(stderr, "\n");
    }
    if (flat) {                                   // egress: the position lists' lengths
        for (int q : {(int)Q_LB4, (int)Q_LB6, (int)Q_CT4, (int)Q_CT6}) {
            fprintf(stderr, "[cv groups] %s %s: largest %u; packets per member position:", what, qn[q],
                    cur[GMAX_WORD0 + q]);
            uint32_t cont = 0;
            for (uint32_t k = 0; k < 16; ++k) {
                if (k + 1 < NPOS) fprintf(stderr, " %u", cur[qcls(q, (int)k)]);
                else cont += cur[qcls(q, (int)k)];
            }
            fprintf(stderr, " %u (the last: groups continued)\n", cont);
        }
        return;
    }
    std::vector<uint32_t> order((size_t)c->gn * 2);
    (void)hipMemcpy(order.data(), c->gorder.p, order.size() * 4, hipMemcpyDeviceToHost);
    const int q4 = flat ? (int)Q_CT4 : (int)Q_NETDEV, q6 = flat ? (int)Q_CT6 : (int)Q_NETDEV6;
    for (int fam = 0; fam < 2; ++fam) {
        const int q = fam ? q6 : q4;
        const DevBuf &wb = fam ? c->gwork6 : c->gwork;
        uint32_t nw = 0;
        uint64_t singles = 0;
        if (flat) {
            nw = cur[qcls(q, 0)];
        } else {
            for (int k = 1; k < NCLASS; ++k) nw += cur[qcls(q, k)];
            singles = cur[SINGLE_WORD0 + q];
        }
        std::vector<uint32_t> w(nw);
        if (nw) (void)hipMemcpy(w.data(), wb.p, (size_t)nw * 4, hipMemcpyDeviceToHost);
        uint64_t hist[33] = {0}, big = 0, pk = 0;
        uint32_t best = 0;
        for (uint32_t e : w) {
            uint32_t sz = 1;
            if (!(e & SINGLE_RUN) && e < order.size()) sz = order[e];
            if (sz == 1) { ++singles; continue; }
            int lg = 0;
            while ((2u << lg) <= sz) ++lg;
            ++hist[lg];
            pk += sz;
            if (sz > 64) big += sz;
            best = std::max(best, sz);
        }
        if (!nw && !singles) continue;
        fprintf(stderr, "[cv groups] %s %s: %llu singletons, %llu packets in runs, largest %u, %llu in runs > 64; "
                "runs by size 2^k:", what, fam ? "v6" : "v4", (unsigned long long)singles, (unsigned long long)pk, best,
                (unsigned long long)big);
        for (int k = 1; k < 33; ++k)
            if (hist[k]) fprintf(stderr, " [%d]%llu", k, (unsigned long long)hist[k]);
        fprintf(stderr, "\n");
    }
}

// Map-API operations on device tables run on the null stream: wait for every batch
// already submitted (on any stream) first, so they see its writes and do not race it.
void drain(cv_ctx *c)
{
    (void)c;
    (void)hipDeviceSynchronize();
}

int ct_io(cv_ctx *c, MapObj *mo, int op, const uint8_t *key, const uint8_t *val, uint8_t *val_out, uint64_t fl)
{
    const bool v6 = mo->kind == MK_CT6;
    drain(c);
    if (op) {
        mo->gen++;
        if (op == 1) mo->live_upper++;
    }
    const uint32_t ks = v6 ? 40 : 14, kw = v6 ? 10 : 4;
    if (!c->ctio.p && c->ctio.alloc(32 * 4)) return -ENOMEM;
    uint32_t io[32] = {0};
    uint8_t kk[40] = {0};
    memcpy(kk, key, ks);
    memcpy(io, kk, kw * 4);
    if (val) memcpy(io + kw, val, 56);
    if (hipMemcpy(c->ctio.p, io, sizeof(io), hipMemcpyHostToDevice) != hipSuccess) return -EIO;
    if (launch_ct_op(mo->ct.view, v6, op, fl, c->ctio.as<uint32_t>(), nullptr)) return -EIO;
    if (hipMemcpy(io, c->ctio.p, sizeof(io), hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
    int rc = (int)io[kw + 16];
    if (!rc && val_out) memcpy(val_out, io + kw, 56);
    return rc;
}

// the live-entry count of a device CT map
int ct_live(cv_ctx *c, MapObj *mo, uint64_t *n)
{
    drain(c);
    return hipMemcpy(n, mo->live.p, 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -EIO;
}

// all (key, value) rows of a device CT table, in slot order (the table's walk order)
int ct_dump(cv_ctx *c, MapObj *mo, std::vector<uint8_t> &keys, std::vector<uint8_t> &vals)
{
    const bool v6 = mo->kind == MK_CT6;
    const uint32_t ks = v6 ? 40 : 14, kw = v6 ? 10 : 4;
    uint64_t live = 0;
    int r = ct_live(c, mo, &live);
    if (r) return r;
    const uint32_t max = (uint32_t)std::min<uint64_t>(live + 64, 0xFFFFFFF0ull);
    DevBuf ds, dk, dv, dc;
    if (ds.alloc((size_t)max * 8) || dk.alloc((size_t)max * kw * 4) || dv.alloc((size_t)max * 64) || dc.alloc(4))
        return -ENOMEM;
    (void)hipMemset(dc.p, 0, 4);
    if (launch_ct_scan(mo->ct.view, v6, mo->ct.nb, ds.as<uint64_t>(), dk.as<uint32_t>(), dv.as<uint32_t>(),
                       dc.as<uint32_t>(), max, nullptr))
        return -EIO;
    uint32_t n = 0;
    (void)hipMemcpy(&n, dc.p, 4, hipMemcpyDeviceToHost);
    if (n > max) return -EIO;                     // the live count lags the table: a bug
    std::vector<uint64_t> slot(n);
    std::vector<uint8_t> kraw((size_t)n * kw * 4), v64((size_t)n * 64);
    if (n) {
        (void)hipMemcpy(slot.data(), ds.p, slot.size() * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(kraw.data(), dk.p, kraw.size(), hipMemcpyDeviceToHost);
        (void)hipMemcpy(v64.data(), dv.p, v64.size(), hipMemcpyDeviceToHost);
    }
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return slot[a] < slot[b]; });
    keys.resize((size_t)n * ks);
    vals.resize((size_t)n * 56);
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t i = ord[j];
        memcpy(&keys[(size_t)j * ks], &kraw[(size_t)i * kw * 4], ks);
        memcpy(&vals[(size_t)j * 56], &v64[(size_t)i * 64], 56);
    }
    return (int)n;
}

// GetNextKey over a device CT map (pkg/bpf/bpf.go:218-245, used by ctmap's dump walk,
// ctmap.go:196-230): the entry after `key` in slot order, the first one when key is
// null or absent (kernel/bpf/hashtab.c htab_map_get_next_key).  The walk reads one
// snapshot of the table, taken once per table generation, so a full walk costs one
// dump plus O(1) per call; slot order is stable across generations (entries never
// move), so a walk that spans batches continues where it was.
// A walk that continues (key = the key the previous call returned) keeps reading its
// snapshot even when batches ran in between: a GetNextKey walk over a changing kernel
// hash map likewise may or may not see entries added or removed meanwhile.  The
// snapshot is retaken when a walk (re)starts -- a null key, or a key that is not the
// one just returned and not in the snapshot -- and the table changed since.  The
// common call (the previous result) is found in O(1) without any index; a key index
// is built only for a walk that jumps.
int ct_next_key(cv_ctx *c, MapObj *mo, const uint8_t *key, uint8_t *next)
{
    const uint32_t ks = mo->kind == MK_CT6 ? 40 : 14;
    const size_t n = mo->snap_keys.size() / ks;
    size_t pos = 0;
    bool found = false;
    if (key && mo->snap_last < n && !memcmp(&mo->snap_keys[mo->snap_last * ks], key, ks)) {
        pos = mo->snap_last + 1;
        found = true;
    } else if (key && mo->snap_gen == mo->gen) {
        if (mo->snap_index.empty() && n) {
            mo->snap_index.reserve(n * 2);
            for (size_t i = 0; i < n; ++i) mo->snap_index.emplace(kstr(&mo->snap_keys[i * ks], ks), i);
        }
        auto it = mo->snap_index.find(kstr(key, ks));
        if (it != mo->snap_index.end()) { pos = it->second + 1; found = true; }
    }
    if (!found && mo->snap_gen != mo->gen) {              // a walk (re)starts on a changed table
        std::vector<uint8_t> vals;
        mo->snap_keys.clear();
        mo->snap_index.clear();
        mo->snap_last = ~(size_t)0;
        const int r = ct_dump(c, mo, mo->snap_keys, vals);
        if (r < 0) return r;
        mo->snap_gen = mo->gen;
        return ct_next_key(c, mo, key, next);
    }
    if (pos >= mo->snap_keys.size() / ks) return -ENOENT;
    memcpy(next, &mo->snap_keys[pos * ks], ks);
    mo->snap_last = pos;
    return 0;
}

// The CT maps a batch may write (every endpoint's CT4 / CT6 map), each once
std::vector<MapObj *> batch_ct_maps(cv_ctx *c)
{
    std::vector<MapObj *> v;
    std::unordered_set<MapObj *> seen;
    for (auto &e : c->eps)
        for (int h : {e.ct4, e.ct6}) {
            MapObj *m = get(c, h);
            if (m && m->kind != MK_PLAIN && seen.insert(m).second) v.push_back(m);
        }
    return v;
}

// The device view of the launch's CT maps (rebuilt when the map list or the endpoints
// change): per map its live-count pointer and max_entries, per endpoint the index of its
// CT4 / CT6 map (ADMIT_NO_MAP: none) -- what the admission walks of any number of maps
// (per-endpoint maps: ConntrackLocal) and the batched live-count reads use.
int map_table(cv_ctx *c, const std::vector<MapObj *> &maps)
{
    if (maps == c->mt_maps && c->mt_eps == c->eps_gen) return 0;
    if (maps.size() >= ADMIT_NO_MAP) return -E2BIG;
    std::unordered_map<const MapObj *, uint16_t> idx;
    std::vector<unsigned long long *> live(maps.size());
    std::vector<unsigned long long> cap(maps.size());
    for (size_t k = 0; k < maps.size(); ++k) {
        idx[maps[k]] = (uint16_t)k;
        live[k] = maps[k]->live.as<unsigned long long>();
        cap[k] = maps[k]->cap;
    }
    std::vector<uint16_t> mi4(c->eps.size() + 1, (uint16_t)ADMIT_NO_MAP), mi6(c->eps.size() + 1, (uint16_t)ADMIT_NO_MAP);
    for (size_t e = 0; e < c->eps.size(); ++e) {
        auto a = idx.find(get(c, c->eps[e].ct4)), b = idx.find(get(c, c->eps[e].ct6));
        if (a != idx.end()) mi4[e] = a->second;
        if (b != idx.end()) mi6[e] = b->second;
    }
    int r = 0;
    if ((r = c->mt_live.upload(live.data(), std::max<size_t>(1, live.size()) * 8)) ||
        (r = c->mt_cap.upload(cap.data(), std::max<size_t>(1, cap.size()) * 8)) ||
        (r = c->mt_epmi4.upload(mi4.data(), mi4.size() * 2)) || (r = c->mt_epmi6.upload(mi6.data(), mi6.size() * 2)) ||
        (r = c->mt_out.alloc(std::max<size_t>(1, maps.size()) * 8)))
        return r;
    c->mt_maps = maps;
    c->mt_eps = c->eps_gen;
    return 0;
}

// every map's exact live count into live_upper (after every batch already submitted, on
// any stream): one gather kernel and one read for many maps
void refresh_live(cv_ctx *c, const std::vector<MapObj *> &maps)
{
    drain(c);
    if (maps.size() > 4 && !map_table(c, maps)) {
        std::vector<unsigned long long> v(maps.size());
        if (!launch_gather_u64(c->mt_live.as<unsigned long long *const>(), c->mt_out.as<unsigned long long>(),
                               (uint32_t)maps.size(), nullptr) &&
            hipMemcpy(v.data(), c->mt_out.p, v.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            for (size_t k = 0; k < maps.size(); ++k) maps[k]->live_upper = v[k];
            return;
        }
    }
    for (MapObj *m : maps) {
        uint64_t v = 0;
        if (hipMemcpy(&v, m->live.p, 8, hipMemcpyDeviceToHost) == hipSuccess) m->live_upper = v;
    }
}

// Many CT maps (ConntrackLocal): whether a launch surely fits every map by a per-map
// bound of its creates (CtBound, cv_dp.hpp) -- the global rule (every map's room >= W n)
// sends every launch over 64 000-entry per-endpoint maps through the admission passes.
// One sync (the flag).  A launch that fits leaves every map's count to be re-read when
// the next launch plans.
bool ct_bound_fits(cv_ctx *c, const DpParams &p, const BatchDev &b, const uint4 *records, uint32_t mode,
                   const uint16_t *src_ep, uint32_t ep0, const std::vector<MapObj *> &cts, hipStream_t s)
{
    if (cts.size() < 2) return false;
    for (MapObj *m : cts)                      // (a full map: the launch is admitted anyway -- ct_fits
        if (m->live_upper >= m->cap) return false;   //  just read the exact counts -- skip the check)
    if (map_table(c, cts)) return false;
    const uint32_t nm = (uint32_t)cts.size();
    const uint64_t s4 = mode == 1 && p.lb4.buckets ? (p.lb4.mask + 1) * Lb4Spec::SPB : 0,
                   s6 = mode == 1 && p.lb6.buckets ? (p.lb6.mask + 1) * Lb6Spec::SPB : 0;
    const size_t bytes = (size_t)nm * 8 + (s4 + s6) * 4 + 64;
    if (c->bnd_buf.n < bytes && c->bnd_buf.alloc(bytes)) return false;
    if (hipMemsetAsync(c->bnd_buf.p, 0, bytes, s) != hipSuccess) return false;
    CtBound bd{};
    bd.bound = c->bnd_buf.as<unsigned long long>();
    bd.svc4 = reinterpret_cast<uint32_t *>(bd.bound + nm);
    bd.svc6 = bd.svc4 + s4;
    bd.flag = bd.svc6 + s6;
    bd.live = c->mt_live.as<unsigned long long *const>();
    bd.cap = c->mt_cap.as<const unsigned long long>();
    bd.epmi4 = c->mt_epmi4.as<const uint16_t>();
    bd.epmi6 = c->mt_epmi6.as<const uint16_t>();
    bd.src_ep = src_ep;
    bd.ep0 = ep0;
    bd.nmaps = nm;
    bd.n_eps = (uint32_t)c->eps.size();
    bd.w_src = 7;                              // (a source program's creates: cv_lxc_egress's W)
    bd.w_dst = 2;                              // (a delivery: the tuple and its ICMP twin)
    bd.mode = mode;
    uint32_t flag[2] = {1u, 0u};
    if (launch_ct_bound(p, b, records, bd, s) ||
        hipMemcpyAsync(flag, bd.flag, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return false;
    c->bound_checks++;
    if (getenv("CV_ADMIT_STATS"))
        fprintf(stderr, "[cv bound] mode %u: %u packets, %u maps, fits %d (unseen %u)\n", mode, b.n, nm, !flag[0],
                flag[1]);
    if (flag[0]) return false;
    c->bound_fits++;
    for (MapObj *m : cts) {
        m->live_upper = m->cap;                // (re-read when the next launch plans)
        m->gen++;
    }
    return true;
}

// Launch-chunk planning against max_entries (ct_live_add, cv_dev.hpp).  A packet
// creates at most W entries in a map (ingress: the tuple and its ICMP-related twin;
// egress: a service create, the connection with its NAT tuple, and the delivery's
// ingress create), so a chunk of n packets fits when every map has W * n free
// entries.  The host keeps an upper bound of each count, raised by W per packet it
// launches, and reads the true counts (one sync) only when a bound gets close.  Next
// to a limit the chunk is one packet with guard = 1: its creates check the count.
uint32_t ct_plan(cv_ctx *c, const std::vector<MapObj *> &maps, uint32_t want, uint32_t W, hipStream_t s,
                 uint32_t *guard)
{
    *guard = 0;
    auto room = [&]() {
        uint64_t r = ~0ull;
        for (MapObj *m : maps) r = std::min(r, m->cap > m->live_upper ? m->cap - m->live_upper : 0);
        return r;
    };
    uint64_t r = room();
    if (r < (uint64_t)W * want) {
        // every batch already submitted, on any stream, has finished (a batch on another
        // stream against the same CT maps holds a reservation this read would drop)
        (void)s;
        refresh_live(c, maps);
        r = room();
    }
    uint64_t n = std::min<uint64_t>(want, r / W);
    if (n == 0) {
        n = 1;
        *guard = 1;
    }
    for (MapObj *m : maps) {
        m->live_upper += W * n;
        m->gen++;
    }
    return (uint32_t)n;
}

// How many of the next n packets (each creating at most W entries per map) surely fit
// every map's room (no reservation); the exact live counts are read (after every batch
// already submitted) when the running upper bound says the n may not fit.
constexpr uint32_t SPLIT_MIN = 1u << 20;
uint32_t ct_fit_count(cv_ctx *c, const std::vector<MapObj *> &maps, uint32_t n, uint32_t W)
{
    auto room = [&]() {
        uint64_t r = ~0ull;
        for (MapObj *m : maps) r = std::min(r, m->cap > m->live_upper ? m->cap - m->live_upper : 0);
        return r;
    };
    if (room() < (uint64_t)W * n) refresh_live(c, maps);
    return (uint32_t)std::min<uint64_t>(n, room() / W);
}

// Whether a launch of n packets (each creating at most W entries per map) surely
// fits every map's room; reads the exact live counts (after every batch already
// submitted) when the running upper bound says it may not.  A launch that fits is
// reserved: the bound rises by W * n.
bool ct_fits(cv_ctx *c, const std::vector<MapObj *> &maps, uint32_t n, uint32_t W)
{
    auto room = [&]() {
        uint64_t r = ~0ull;
        for (MapObj *m : maps) r = std::min(r, m->cap > m->live_upper ? m->cap - m->live_upper : 0);
        return r;
    };
    if (room() < (uint64_t)W * n) {
        refresh_live(c, maps);
        if (room() < (uint64_t)W * n) return false;
    }
    for (MapObj *m : maps) {
        m->live_upper += (uint64_t)W * n;
        m->gen++;
    }
    return true;
}

// A netdev launch next to max_entries, exact (cv_kernels.hip "conntrack admission"):
// the front and the grouping once, then windows.  A window repeats k_ct_intent + the
// budget scans over every packet not yet run until the intents stop changing (each
// pass reads the previous one's budgets for creates of earlier group members: the
// fixed point is the sequential answer), then runs the conntrack stages over it.  A
// window ends early at a packet whose run changed more keys than Changed holds, or,
// after MAX_PASSES, just past the last packet the passes have settled.  One host read
// per pass (three words).
int run_admitted(cv_ctx *c, DpParams p, const BatchDev &bc, const OutDev &oc, uint32_t now, int with_prefilter,
                 const GroupScratch &gs, const std::vector<MapObj *> &cts, hipStream_t s)
{
    constexpr int MAX_PASSES = 12;
    const uint32_t n = bc.n;
    int r = map_table(c, cts);
    if (r) return r;
    Admit a{};
    a.nmaps = (uint32_t)cts.size();
    a.live = c->mt_live.as<unsigned long long *const>();
    a.cap = c->mt_cap.as<const unsigned long long>();
    a.ep_mi4 = c->mt_epmi4.as<const uint16_t>();
    a.ep_mi6 = c->mt_epmi6.as<const uint16_t>();
    size_t sort_bytes = 0;
    if (sort_keys64(nullptr, &sort_bytes, nullptr, nullptr, n, 48, nullptr)) return -EIO;
    if ((c->adm_ib.n < (size_t)n * 2 && c->adm_ib.alloc((size_t)n * 2)) ||
        (c->adm_mi.n < (size_t)n * 2 && c->adm_mi.alloc((size_t)n * 2)) ||
        (c->adm_keys.n < (size_t)n * 16 && c->adm_keys.alloc((size_t)n * 16)) ||
        (c->adm_sort.n < sort_bytes && c->adm_sort.alloc(sort_bytes)) ||
        (c->adm_evt.n < (size_t)n * 128 &&
         (c->adm_evt.alloc((size_t)n * 128) || hipMemset(c->adm_evt.p, 0, c->adm_evt.n) != hipSuccess)) ||
        (!c->adm_tsum.p && c->adm_tsum.alloc((size_t)4096 * 12)) || (!c->adm_win.p && c->adm_win.alloc(32)))
        return -ENOMEM;
    a.ib = c->adm_ib.as<uint8_t>();
    a.budget = a.ib + n;
    a.mi = c->adm_mi.as<uint16_t>();
    a.keys = c->adm_keys.as<unsigned long long>();
    a.keys_sorted = a.keys + n;
    a.sort_tmp = c->adm_sort.p;
    a.sort_bytes = c->adm_sort.n;
    a.tsum = c->adm_tsum.as<uint32_t>();
    a.hi = c->adm_win.as<uint32_t>();
    a.evt = c->adm_evt.as<unsigned long long>();
    const char *inj = getenv("CV_ADMIT_INJECT");
    a.inject = inj ? (uint32_t)strtoul(inj, nullptr, 0) : ~0u;
    r = launch_netdev_front(p, bc, with_prefilter, oc, gs, s);
    if (r) return r;
    // packets that reach no conntrack stage keep 0 (no creates, no deletes, map 0);
    // k_ct_intent rewrites the others every pass.  The first pass assumes that earlier
    // creates fail (budget 0).
    if (hipMemsetAsync(a.ib, 0, (size_t)n * 2, s) != hipSuccess) return -EIO;
    const bool stats = getenv("CV_ADMIT_STATS") != nullptr;
    uint32_t windows = 0, passes = 0;
    for (uint32_t lo = 0; lo < n; ++windows) {
        a.lo = lo;
        uint32_t end = lo, w[5] = {n, n, n, 0, 0};
        for (int pass = 0;; ++pass) {
            a.pass = (uint32_t)pass;
            if (++c->adm_stamp == 0) {                            // (2^32 passes: stale stamps cleared)
                (void)hipMemsetAsync(c->adm_evt.p, 0, c->adm_evt.n, s);
                c->adm_stamp = 1;
            }
            a.stamp = c->adm_stamp;
            if ((r = launch_admission(p, bc, gs, a, s))) return r;
            ++passes;
            hipError_t e = hipMemcpyAsync(w, a.hi, 20, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                fprintf(stderr, "[cv] admission pass at %u: %s\n", lo, hipGetErrorString(e));
                return -EIO;
            }
            if (w[3]) {                                           // a stale or corrupt intent byte
                fprintf(stderr, "[cv] admission pass at %u: intent error %#x\n", lo, w[3]);
                return -EPROTO;
            }
            if ((r = launch_admission_walks(bc, a, w[4], s))) return r;   // (the budgets, in stream order)
            const uint32_t hi = w[0], chg = w[1], used = w[2];
            if (hi <= lo || hi > n || (pass && chg <= lo) || used <= lo) {   // (the window's first packet is exact)
                fprintf(stderr, "[cv] admission window at %u: %u %u %u of %u\n", lo, hi, chg, used, n);
                return -EPROTO;
            }
            // exact: every packet before the first that read a budget (pass 0), or, once
            // the budgets come from the previous pass, up to the first that changed
            if (used >= hi || (pass && chg >= hi)) { end = hi; break; }
            if (pass + 1 == MAX_PASSES) { end = pass ? std::max(chg + 1, used) : used; break; }
        }
        if (stats && end < n) {                                   // why the window ends
            uint8_t why = 0;
            (void)hipMemcpy(&why, a.ib + end, 1, hipMemcpyDeviceToHost);
            fprintf(stderr, "[cv admit] window [%u, %u) (%u passes so far): %s\n", lo, end, passes,
                    (why & 64) ? "too many changed keys in a run" : "intents still changing");
        }
        DpParams pw = p;
        pw.win_lo = lo;
        pw.win_span = end - lo;
        pw.budget = a.budget;
        if ((r = launch_netdev_stages(pw, bc, now, oc, gs, s))) return r;
        lo = end;
    }
    for (MapObj *m : cts) {
        m->live_upper = m->cap;                                   // (re-read when the next launch plans)
        m->gen++;
    }
    if (stats) fprintf(stderr, "[cv admit] %u packets in %u windows, %u passes\n", n, windows, passes);
    return 0;
}

// An egress launch next to max_entries, exact (cv_kernels.hip "egress admission"): the
// whole pipeline runs with per-packet budgets of CT creates, and the budget scan then
// tells whether every packet got the creates the sequential run gives it.  If not, the
// device state the pass wrote (the CT maps, the policy counters, the metrics, the event
// rings' counts) goes back to the copy taken before the first pass and the pipeline runs
// again with the scan's budgets.  The first pass gives every packet 7 (none if a map is
// full): a launch that crosses max_entries settles in two passes, one that starts full in
// one.  One host read per pass (one word).  Needs one CT4 and at most one CT6 map.
bool egress_admissible(const std::vector<MapObj *> &cts)
{
    int n4 = 0, n6 = 0;
    for (MapObj *m : cts) (m->kind == MK_CT4 ? n4 : n6)++;
    return n4 <= 1 && n6 <= 1;
}

int lxc_admitted(cv_ctx *c, const DpParams &p, const BatchDev &bc, const uint16_t *src_ep, uint32_t ep0,
                 const uint32_t *flow_hash, uint32_t now, const OutDev &oc, const std::vector<MapObj *> &cts,
                 hipStream_t s)
{
    const int MAX_PASSES = c->hk.eadm_max_passes;              // (8; tests of the fallback lower it)
    const uint32_t n = bc.n;
    // the state a pass writes, and where its copy goes
    struct Region { void *src; size_t bytes, off; };
    std::vector<Region> regs;
    size_t total = 0;
    auto add = [&](void *src, size_t bytes) {
        if (!src || !bytes) return;
        regs.push_back(Region{src, bytes, total});
        total += (bytes + 255) & ~(size_t)255;
    };
    MapObj *map_of[2] = {nullptr, nullptr};
    for (MapObj *m : cts) map_of[m->kind == MK_CT4 ? 0 : 1] = m;
    size_t live_off[2] = {0, 0};
    add(c->metrics, METRICS_WORDS * 8);
    for (int k = 0; k < 2; ++k)
        if (MapObj *m = map_of[k]) {
            live_off[k] = total;
            add(m->live.p, 8);
            add(m->ct.buckets.p, m->ct.buckets.n);
            add(m->ct.vals.p, m->ct.vals.n);
            add(m->ct.aux.p, m->ct.aux.n);
        }
    std::set<const void *> seen;
    for (auto &e : c->eps) {
        MapObj *m = get(c, e.policy);
        if (m && seen.insert(m->pol.vals.p).second) {
            add(m->pol.vals.p, m->pol.vals.n);
            add(m->pol.aux.p, m->pol.aux.n);
        }
    }
    add(c->notify_count, 4);
    add(c->trace_count, 4);
    if (c->eadm_save.n < total) {                                 // a copy that would crowd the device out:
        size_t fr = 0, all = 0;                                   // the caller's planned launches instead
        if (hipMemGetInfo(&fr, &all) != hipSuccess || total > fr / 2) return -ENOMEM;
    }
    if ((c->eadm_save.n < total && c->eadm_save.alloc(total)) ||
        (c->eadm_buf.n < (size_t)n * 4 + 2 * 4096 * 8 + 256 && c->eadm_buf.alloc((size_t)n * 4 + 2 * 4096 * 8 + 256)))
        return -ENOMEM;
    uint8_t *save = c->eadm_save.as<uint8_t>();
    for (const Region &g : regs)
        if (hipMemcpyAsync(save + g.off, g.src, g.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return -EIO;
    uint8_t *buf = c->eadm_buf.as<uint8_t>();
    EAdmit a{};
    a.n = n;
    a.intent = buf;
    uint8_t *bud[2] = {buf + n, buf + 2 * (size_t)n};
    uint8_t *left = buf + 3 * (size_t)n;
    a.tsum = reinterpret_cast<uint32_t *>(buf + ((4 * (size_t)n + 255) & ~(size_t)255));
    a.flag = a.tsum + 2 * 4096 * 2;
    bool full = true;                                             // (the live counts: exact, read by ct_fits)
    for (int k = 0; k < 2; ++k) {
        a.live0[k] = reinterpret_cast<const unsigned long long *>(save + live_off[k]);   // (absent: cap 0, no room)
        a.cap[k] = map_of[k] ? map_of[k]->cap : 0;
        if (map_of[k] && map_of[k]->live_upper < map_of[k]->cap) full = false;
    }
    // the first pass: 7 creates per packet, or none when every map is full
    if (hipMemsetAsync(bud[0], full ? 0 : 7, n, s) != hipSuccess) return -EIO;
    const bool stats = getenv("CV_ADMIT_STATS") != nullptr;
    int cur = 0, pass = 0;
    for (;; ++pass) {
        DpParams pp = p;
        pp.budget = bud[cur];
        pp.eg_left = left;
        pp.eg_intent = const_cast<uint8_t *>(a.intent);
        GroupScratch gs = next_groups(c, 3, s);
        gs.gbits = gbin_bits(n);
        int r = launch_lxc_egress(pp, bc, src_ep, ep0, flow_hash, now, oc, gs, s);
        if (r) return r;
        a.used = bud[cur];
        a.next = bud[cur ^ 1];
        if ((r = launch_egress_admission(a, s))) return r;
        uint32_t flag = 0;
        hipError_t e = hipMemcpyAsync(&flag, a.flag, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            fprintf(stderr, "[cv] egress admission pass %d: %s\n", pass, hipGetErrorString(e));
            return -EIO;
        }
        if (!flag) break;                                         // the sequential run
        for (const Region &g : regs)                              // back to the state before the window
            if (hipMemcpyAsync(g.src, save + g.off, g.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return -EIO;
        if (pass + 1 == MAX_PASSES) {
            fprintf(stderr, "[cv] egress admission: no fixed point after %d passes (%u packets)\n", MAX_PASSES, n);
            return -EAGAIN;
        }
        cur ^= 1;
    }
    for (MapObj *m : cts) {
        m->live_upper = m->cap;                                   // (re-read when the next launch plans)
        m->gen++;
    }
    if (stats) fprintf(stderr, "[cv admit] egress: %u packets, %d passes\n", n, pass + 1);
    return 0;
}

// Egress next to max_entries with any number of CT maps (ConntrackLocal: every endpoint
// its own CT4 / CT6 map), exact.  As lxc_admitted, a pass runs the whole pipeline with
// budgets and the budget scan tells whether it was the sequential run; here a packet has
// two budgets -- its source program's creates go to its source endpoint's map, its local
// delivery's to the destination's -- and every map's walk is one segment of a scan over
// the (map, packet, slot) elements, sorted (launch_eam_*).  A pass that was not the
// sequential run is undone without a copy of the maps: each CT slot the pass wrote was
// saved before its first write (Snap: copy-on-first-write into a set sized for 8 written
// slots per packet, cv_dev.hpp snap_slot), the live counts, the metrics, the policy values
// and the event rings' counts were copied before the first pass.  Launches of at most
// EAM_WINDOW packets; -EAGAIN (no fixed point, state restored) and -ENOMEM (no room for the
// set, nothing ran) send the caller to planned launches.
constexpr uint32_t EAM_WINDOW = 1u << 23;
// `launch` runs one pass of the n packets (the egress pipeline, or a delivery launch of n
// records: cv_lxc_deliver).  `front`: the pass's first kernel resets every packet's
// intents and loads its budgets (k_egress_front); otherwise (deliveries: slot 1 only)
// the host does before each pass.
int lxc_admitted_maps(cv_ctx *c, const DpParams &p, uint32_t n, const uint16_t *src_ep, uint32_t ep0,
                      const std::vector<MapObj *> &cts, hipStream_t s,
                      const std::function<int(const DpParams &)> &launch, bool front, const char *what, int v6 = 0)
{
    const int MAX_PASSES = c->hk.eadm_max_passes;
    if (n > EAM_WINDOW) return -EINVAL;
    int r = map_table(c, cts);
    if (r) return r;
    const uint32_t nm = (uint32_t)cts.size();
    // the state besides the CT slots, copied once
    struct Region { void *src; size_t bytes, off; };
    std::vector<Region> regs;
    size_t total = 0;
    auto add = [&](void *src, size_t bytes) {
        if (!src || !bytes) return;
        regs.push_back(Region{src, bytes, total});
        total += (bytes + 255) & ~(size_t)255;
    };
    add(c->metrics, METRICS_WORDS * 8);
    std::set<const void *> seen;
    for (auto &e : c->eps) {
        MapObj *m = get(c, e.policy);
        if (m && seen.insert(m->pol.vals.p).second) {
            add(m->pol.vals.p, m->pol.vals.n);
            add(m->pol.aux.p, m->pol.aux.n);
        }
    }
    add(c->notify_count, 4);
    add(c->trace_count, 4);
    const uint64_t scap = (uint64_t)n * SNAP_PER;                 // (a packet writes <= 6 slots)
    size_t sort_bytes = 0;
    if (sort_keys64(nullptr, &sort_bytes, nullptr, nullptr, 2 * n, 48, nullptr)) return -EIO;
    const size_t nb = (size_t)n, live_off = ((10 * nb + 255) & ~(size_t)255);
    const size_t buf_bytes = live_off + (size_t)nm * 8 + 4096 * 12 + 256;
    const size_t snap_bytes = scap * SNAP_U4 * 16 + nb;           // (+ the per-packet entry counts)
    if (c->eam_snap.n < snap_bytes || c->eadm_save.n < total) {
        size_t fr = 0, all = 0;                                   // (a set that would crowd the device out:
        if (hipMemGetInfo(&fr, &all) != hipSuccess || snap_bytes + total > fr / 2) return -ENOMEM;   // planned)
    }
    if ((c->eadm_save.n < total && c->eadm_save.alloc(total)) ||
        (c->eam_buf.n < buf_bytes && c->eam_buf.alloc(buf_bytes)) ||
        (c->eam_keys.n < (size_t)n * 32 + sort_bytes && c->eam_keys.alloc((size_t)n * 32 + sort_bytes)) ||
        (c->eam_snap.n < snap_bytes && c->eam_snap.alloc(snap_bytes)) ||
        (c->eadm_buf.n < 128 && c->eadm_buf.alloc(128)))
        return -ENOMEM;
    uint8_t *save = c->eadm_save.as<uint8_t>();
    for (const Region &g : regs)
        if (hipMemcpyAsync(save + g.off, g.src, g.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return -EIO;
    uint8_t *buf = c->eam_buf.as<uint8_t>();
    uint8_t *intent = buf, *intent2 = buf + nb, *left = buf + 2 * nb, *left2 = buf + 3 * nb;
    uint8_t *bud[2] = {buf + 4 * nb, buf + 6 * nb};               // (2n each: slot 0, then slot 1)
    uint16_t *dst = reinterpret_cast<uint16_t *>(buf + 8 * nb);  // (per packet the delivery's endpoint)
    unsigned long long *live0 = reinterpret_cast<unsigned long long *>(buf + live_off);
    EAdmitM a{};
    a.n = n;
    a.nmaps = nm;
    a.intent = intent;
    a.intent2 = intent2;
    a.src_ep = src_ep;
    a.ep0 = ep0;
    a.ep_mi4 = c->mt_epmi4.as<const uint16_t>();
    a.ep_mi6 = c->mt_epmi6.as<const uint16_t>();
    a.n_eps = (uint32_t)c->eps.size();
    a.live0 = live0;
    a.cap = c->mt_cap.as<const unsigned long long>();
    a.keys = c->eam_keys.as<unsigned long long>();
    a.keys_sorted = a.keys + 2 * nb;
    a.sort_tmp = a.keys + 4 * nb;
    a.sort_bytes = sort_bytes;
    a.tsum = reinterpret_cast<uint32_t *>(buf + live_off + (size_t)nm * 8);
    a.cnt = c->eadm_buf.as<uint32_t>();
    a.dst_ep = dst;
    Snap sn{};
    sn.log = c->eam_snap.as<uint4>();
    sn.cnt = reinterpret_cast<uint8_t *>(sn.log + scap * SNAP_U4);
    sn.n = c->hk.snap_ablate ? 0u : n;                            // (timing only: no slot saved, wrong undo)
    sn.err = a.cnt + 4;
    if ((r = launch_gather_u64(c->mt_live.as<unsigned long long *const>(), live0, nm, s))) return r;
    a.next = bud[0];
    a.next2 = bud[0] + nb;
    if ((r = launch_eam_first(a, s))) return r;
    const bool stats = getenv("CV_ADMIT_STATS") != nullptr;
    int cur = 0, pass = 0;
    for (;; ++pass) {
        c->eam_snap_host[pass & 1] = sn;                          // (the async copy's source outlives the call)
        if (hipMemsetAsync(a.cnt, 0, 32, s) != hipSuccess || hipMemsetAsync(sn.cnt, 0, nb, s) != hipSuccess ||
            hipMemcpyAsync(a.cnt + 8, &c->eam_snap_host[pass & 1], sizeof(Snap), hipMemcpyHostToDevice, s) != hipSuccess)
            return -EIO;
        DpParams pp = p;
        pp.budget = bud[cur];
        pp.eg_left = left;
        pp.eg_intent = intent;
        pp.eg_left2 = left2;
        pp.eg_intent2 = intent2;
        pp.eg_dst = dst;
        pp.snap = reinterpret_cast<const Snap *>(a.cnt + 8);
        if (!front &&                                             // (slot 1 only: no source program ran; the
            (hipMemsetAsync(intent, v6 ? 16 : 0, nb, s) != hipSuccess ||   //  family bit of the intent byte)
             hipMemsetAsync(intent2, 0, nb, s) != hipSuccess || hipMemsetAsync(left, 0, nb, s) != hipSuccess ||
             hipMemsetAsync(dst, 0xFF, 2 * nb, s) != hipSuccess ||
             hipMemcpyAsync(left2, bud[cur] + nb, nb, hipMemcpyDeviceToDevice, s) != hipSuccess))
            return -EIO;
        if ((r = launch(pp))) {
            if (sn.n) (void)launch_snap_clear(sn, s);
            return r;
        }
        a.used = bud[cur];
        a.used2 = bud[cur] + nb;
        a.next = bud[cur ^ 1];
        a.next2 = bud[cur ^ 1] + nb;
        if (hipMemcpyAsync(a.next, a.used, 2 * nb, hipMemcpyDeviceToDevice, s) != hipSuccess) return -EIO;
        if ((r = launch_eam_keys(a, s))) return r;
        uint32_t w[8] = {};
        hipError_t e = hipMemcpyAsync(w, a.cnt, 32, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            fprintf(stderr, "[cv] egress admission pass %d: %s\n", pass, hipGetErrorString(e));
            return -EIO;
        }
        if (w[2]) {
            fprintf(stderr, "[cv] egress admission pass %d: a create in a CT map outside the launch's\n", pass);
            if (sn.n) (void)launch_snap_clear(sn, s);             // (no slot bit outlives the pass)
            return -EPROTO;
        }
        if ((r = launch_eam_walks(a, w[0], s))) return r;
        const uint32_t K = w[0];
        if (sn.n && (r = launch_snap_clear(sn, s))) return r;    // (the slots' bits, before the next pass)
        e = hipMemcpyAsync(w, a.cnt, 32, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return -EIO;
        if (stats) fprintf(stderr, "[cv admit] %s pass %d: %u elements, %u not sequential (first packet %d)\n",
                           what, pass, K, w[1], w[1] ? (int)w[3] : -1);
        if (!w[1]) break;                                         // the sequential run
        if (w[4]) {                                               // (cannot be undone: never with <= 8 slots per packet)
            fprintf(stderr, "[cv] egress admission pass %d: slot set full (%llu entries)\n", pass,
                    (unsigned long long)scap);
            return -EIO;
        }
        if ((sn.n && (r = launch_snap_restore(sn, s))) ||         // back to the state before the window
            (r = launch_scatter_u64(c->mt_live.as<unsigned long long *const>(), live0, nm, s)))
            return r;
        for (const Region &g : regs)
            if (hipMemcpyAsync(g.src, save + g.off, g.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return -EIO;
        if (pass + 1 == MAX_PASSES) {
            fprintf(stderr, "[cv] egress admission: no fixed point after %d passes (%u packets, %u maps)\n",
                    MAX_PASSES, n, nm);
            return -EAGAIN;
        }
        cur ^= 1;
    }
    for (MapObj *m : cts) {
        m->live_upper = m->cap;                                   // (re-read when the next launch plans)
        m->gen++;
    }
    if (stats) fprintf(stderr, "[cv admit] %s: %u packets, %d passes, %u maps\n", what, n, pass + 1, nm);
    return 0;
}

// live policy counters of one key from HBM (device-authoritative)
void policy_counters(MapObj *mo, const uint8_t *key, uint8_t *val)
{
    if (!mo->is_policy || !mo->pol.view.buckets || mo->written.count(kstr(key, 8))) return;
    if (mo->pol_version != mo->hm->version) {
        // the table was not recompiled since the last write; slots of unchanged keys
        // are still those of the image
    }
    HashTable img{mo->pol.hb.data(), nullptr, mo->pol.nb - 1, 32, PolicySpec::SPB};
    uint32_t kw[2] = {rd32(key), rd32(key + 4)};
    int64_t s = host_find<PolicySpec>(img, kw);
    if (s < 0) return;
    uint8_t v[32];
    if (hipMemcpy(v, mo->pol.vals.as<uint8_t>() + (size_t)s * 32, 32, hipMemcpyDeviceToHost) == hipSuccess)
        memcpy(val + 8, v + 8, 16);
}

}  // namespace

// ================================================== the node view (cv_node.hpp)
namespace cv {

int node_view(cv_ctx *c, NodeView &v)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    v.eps.clear();
    v.svc.clear();
    for (const Endpoint &e : c->eps) {
        NodeEndpoint ne{};
        ne.ipv4 = e.ipv4;
        memcpy(ne.ipv6, e.ipv6, 16);
        ne.ct4 = e.ct4;
        ne.ct6 = e.ct6;
        v.eps.push_back(ne);
    }
    // the slave entries (slave != 0) of the service maps name the backends (lb.h:43-81)
    for (int fam = 0; fam < 2; ++fam) {
        MapObj *m = get(c, c->role[fam ? CV_ROLE_LB6_SERVICES : CV_ROLE_LB4_SERVICES]);
        if (!m) continue;
        const uint32_t alen = fam ? 16 : 4;
        m->hm->for_each([&](const uint8_t *k, const uint8_t *val) {
            if (!(k[alen + 2] | k[alen + 3])) return;
            NodeService ns{};
            ns.v6 = (uint8_t)fam;
            memcpy(ns.vip, k, alen);
            memcpy(ns.backend, val, alen);
            memcpy(&ns.vport, k + alen, 2);
            memcpy(&ns.bport, val + alen, 2);
            v.svc.push_back(ns);
        });
    }
    v.loopback = c->node.ipv4_loopback;
    return 0;
}

int node_key(cv_ctx *c, NodeKey &k)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    k = NodeKey{};
    k.uid = c->uid;
    k.eps = c->eps_gen;
    for (int fam = 0; fam < 2; ++fam) {
        const int h = c->role[fam ? CV_ROLE_LB6_SERVICES : CV_ROLE_LB4_SERVICES];
        MapObj *m = get(c, h);
        k.lb[2 * fam] = (uint64_t)(int64_t)h;
        k.lb[2 * fam + 1] = m ? m->hm->version : 0;
    }
    k.loopback = c->node.ipv4_loopback;
    return 0;
}

int ct_counts(cv_ctx *c, const std::vector<int> &handles, std::vector<uint64_t> &live, std::vector<uint64_t> &cap)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    std::vector<MapObj *> ms;
    for (int h : handles) {
        MapObj *m = get(c, h);
        if (!m) return -EBADF;
        ms.push_back(m);
    }
    if (c->device < 0) {                                          // (host-only context: the host store)
        live.resize(ms.size());
        cap.resize(ms.size());
        for (size_t k = 0; k < ms.size(); ++k) {
            live[k] = ms[k]->hm->count();
            cap[k] = ms[k]->hm->max_entries;
        }
        return 0;
    }
    if (set_device(c)) return -ENODEV;
    for (MapObj *m : ms)
        if (m->kind == MK_PLAIN) return -EINVAL;
    refresh_live(c, ms);
    live.resize(ms.size());
    cap.resize(ms.size());
    for (size_t k = 0; k < ms.size(); ++k) {
        live[k] = ms[k]->live_upper;
        cap[k] = ms[k]->cap;
    }
    return 0;
}

}  // namespace cv

// ======================================================================= C-ABI
extern "C" {

const char *cv_version(void) { return "cilium_hip 0.1.0 gfx950"; }

int cv_open(int hip_device, cv_ctx **out)
{
    if (!out) return -EINVAL;
    static std::atomic<uint64_t> uids{0};
    cv_ctx *c = new cv_ctx();
    c->uid = ++uids;
    c->device = hip_device;
    c->hk.read();
    for (int r = 0; r < CV_NUM_ROLES; ++r) { c->role[r] = -1; c->role_version[r] = 0; }
    if (hip_device == -1) {                 // host-only context: map store without a device
        *out = c;
        return 0;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || hip_device < 0 || hip_device >= n) { delete c; return -ENODEV; }
    if (set_device(c)) { delete c; return -ENODEV; }
    if (c->metrics_own.alloc(METRICS_WORDS * 8)) { delete c; return -ENOMEM; }
    (void)hipMemset(c->metrics_own.p, 0, METRICS_WORDS * 8);
    c->metrics = c->metrics_own.as<unsigned long long>();
    void *eh = nullptr;
    if (hipHostMalloc(&eh, 64, hipHostMallocMapped) != hipSuccess) { delete c; return -ENOMEM; }
    c->gerr_host = static_cast<uint32_t *>(eh);
    *c->gerr_host = 0;
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&c->gerr_dev), eh, 0) != hipSuccess) {
        (void)hipHostFree(eh);
        delete c;
        return -ENOMEM;
    }
    if (const char *e = getenv("CV_MAX_CHUNK")) {
        const unsigned long v = strtoul(e, nullptr, 0);
        if (v >= 1 && v <= MAX_CHUNK) c->chunk = (uint32_t)v;
    }
    *out = c;
    return 0;
}

void cv_close(cv_ctx *c)
{
    if (!c) return;
    if (c->device >= 0) {
        (void)hipSetDevice(c->device);
        (void)hipDeviceSynchronize();
        for (Staging &x : c->staging) {
            (void)hipHostFree(x.host);
            (void)hipFree(x.dev);
            (void)hipEventDestroy(x.done);
        }
        if (c->last_ev) (void)hipEventDestroy(c->last_ev);
        if (c->gerr_host) (void)hipHostFree(c->gerr_host);
    }
    delete c;
}

int cv_set_flags(cv_ctx *c, uint32_t flags)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->flags = flags;
    return 0;
}

int cv_map_create(cv_ctx *c, int type, uint32_t ks, uint32_t vs, uint32_t max_entries, uint32_t flags, int *handle)
{
    if (!c || !handle) return -EINVAL;
    if (type != CV_MAP_HASH && type != CV_MAP_LRU_HASH && type != CV_MAP_LPM_TRIE && type != CV_MAP_PERCPU_HASH)
        return -EINVAL;
    if (!ks || !vs || !max_entries || ks > 256) return -EINVAL;
    if (type == CV_MAP_LPM_TRIE && (ks <= 4 || ks > 4 + 256 / 8 * 8 || !(flags & 1))) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    auto mo = std::make_unique<MapObj>();
    mo->hm = std::make_unique<HostMap>(type, ks, vs, max_entries, flags);
    c->maps.push_back(std::move(mo));
    *handle = (int)c->maps.size() - 1;
    return 0;
}

int cv_map_close(cv_ctx *c, int h)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    for (int r = 0; r < CV_NUM_ROLES; ++r) if (c->role[r] == h) return -EBUSY;
    for (auto &e : c->eps) if (e.policy == h || e.ct4 == h || e.ct6 == h) return -EBUSY;
    if (c->device >= 0) (void)hipDeviceSynchronize();
    c->maps[h].reset(new MapObj());
    c->maps[h]->hm.reset(new HostMap(CV_MAP_HASH, 1, 1, 1, 0));
    c->eps_gen++;                              // (a new map object may take the freed one's address)
    return 0;
}

int cv_map_update(cv_ctx *c, int h, const void *key, const void *val, uint64_t fl)
{
    if (!c || !key || !val) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        return ct_io(c, m, 1, (const uint8_t *)key, (const uint8_t *)val, nullptr, fl);
    }
    int r = m->hm->update((const uint8_t *)key, (const uint8_t *)val, fl);
    if (!r && m->is_policy) m->written.insert(kstr((const uint8_t *)key, 8));
    return r;
}

int cv_map_update_batch(cv_ctx *c, int h, const void *keys, const void *vals, uint32_t n, uint64_t fl, uint32_t *done)
{
    if (!c || (n && (!keys || !vals))) return -EINVAL;
    MapObj *m;
    {
        std::lock_guard<std::mutex> g(c->mu);
        m = get(c, h);
        if (!m) return -EBADF;
    }
    const uint8_t *k = (const uint8_t *)keys, *v = (const uint8_t *)vals;
    for (uint32_t i = 0; i < n; ++i) {
        int r = cv_map_update(c, h, k + (size_t)i * m->hm->ks, v + (size_t)i * m->hm->vs, fl);
        if (r) { if (done) *done = i; return r; }
    }
    if (done) *done = n;
    return 0;
}

int cv_map_lookup(cv_ctx *c, int h, const void *key, void *val)
{
    if (!c || !key || !val) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        return ct_io(c, m, 0, (const uint8_t *)key, nullptr, (uint8_t *)val, 0);
    }
    const uint8_t *v = m->hm->lookup((const uint8_t *)key);
    if (!v) return -ENOENT;
    memcpy(val, v, m->hm->vs);
    if (m->is_policy && !set_device(c)) {
        drain(c);
        policy_counters(m, (const uint8_t *)key, (uint8_t *)val);
    }
    return 0;
}

int cv_map_delete(cv_ctx *c, int h, const void *key)
{
    if (!c || !key) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        return ct_io(c, m, 2, (const uint8_t *)key, nullptr, nullptr, 0);
    }
    int r = m->hm->remove((const uint8_t *)key);
    if (!r && m->is_policy) m->written.erase(kstr((const uint8_t *)key, 8));
    return r;
}

// ctmap.GC with GCFilterByTime / ctmap.Flush (pkg/maps/ctmap/ctmap.go:325-432,
// doFiltering :400-408): delete every entry of CT map h whose lifetime is below
// `time`.  A bound (device-resident) CT map is swept on the GPU in one pass; an
// unbound one in its host store.
int cv_ct_gc(cv_ctx *c, int h, uint32_t time, uint32_t *deleted)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    uint32_t n = 0;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        drain(c);
        m->gen++;
        DevBuf d;
        if (d.alloc(8)) return -ENOMEM;
        if (hipMemset(d.p, 0, 8) != hipSuccess) return -EIO;
        if (launch_ct_gc(m->ct.view, m->kind == MK_CT6, m->ct.nb, time, d.as<uint32_t>(), nullptr)) return -EIO;
        if (hipMemcpy(&n, d.p, 4, hipMemcpyDeviceToHost) != hipSuccess) return -EIO;
    } else {
        HostMap *hm = m->hm.get();
        if ((hm->ks != 14 && hm->ks != 40) || hm->vs != 56) return -EINVAL;
        std::vector<std::vector<uint8_t>> dead;
        hm->for_each([&](const uint8_t *k, const uint8_t *v) {
            uint32_t life;
            memcpy(&life, v + 32, 4);
            if (life < time) dead.emplace_back(k, k + hm->ks);
        });
        for (auto &k : dead)
            if (!hm->remove(k.data())) ++n;
    }
    if (deleted) *deleted = n;
    return 0;
}

// slot occupancy of a device CT map: out[0] empty, out[1] dead (tombstones), out[2] live
int cv_ct_slots(cv_ctx *c, int h, uint64_t out[3])
{
    if (!c || !out) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind == MK_PLAIN) return -EINVAL;
    if (set_device(c)) return -ENODEV;
    drain(c);
    DevBuf d;
    if (d.alloc(24)) return -ENOMEM;
    if (hipMemset(d.p, 0, 24) != hipSuccess) return -EIO;
    if (launch_ct_tags(m->ct.view, m->kind == MK_CT6, m->ct.nb, d.as<unsigned long long>(), nullptr)) return -EIO;
    return hipMemcpy(out, d.p, 24, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -EIO;
}

int cv_map_get_next_key(cv_ctx *c, int h, const void *key, void *next)
{
    if (!c || !next) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        return ct_next_key(c, m, (const uint8_t *)key, (uint8_t *)next);
    }
    return m->hm->next_key((const uint8_t *)key, (uint8_t *)next);
}

int cv_map_count(cv_ctx *c, int h, uint32_t *count)
{
    if (!c || !count) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    if (m->kind != MK_PLAIN) {
        if (set_device(c)) return -ENODEV;
        uint64_t n = 0;
        const int r = ct_live(c, m, &n);
        *count = (uint32_t)n;
        return r;
    }
    *count = m->hm->count();
    return 0;
}

int cv_map_dump(cv_ctx *c, int h, void *keys, void *vals, uint32_t max)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *m = get(c, h);
    if (!m) return -EBADF;
    const uint32_t ks = m->hm->ks, vs = m->hm->vs;
    if (m->kind != MK_PLAIN) {
        std::vector<uint8_t> kb, vb;
        if (set_device(c)) return -ENODEV;
        int n = ct_dump(c, m, kb, vb);
        if (n < 0) return n;
        uint32_t w = std::min<uint32_t>((uint32_t)n, max);
        if (keys) memcpy(keys, kb.data(), (size_t)w * ks);
        if (vals) memcpy(vals, vb.data(), (size_t)w * vs);
        return (int)w;
    }
    uint32_t w = 0;
    if (m->is_policy && !set_device(c)) drain(c);
    m->hm->for_each([&](const uint8_t *k, const uint8_t *v) {
        if (w >= max) return;
        if (keys) memcpy((uint8_t *)keys + (size_t)w * ks, k, ks);
        if (vals) {
            uint8_t *dst = (uint8_t *)vals + (size_t)w * vs;
            memcpy(dst, v, vs);
            if (m->is_policy) policy_counters(m, k, dst);
        }
        w++;
    });
    return (int)w;
}

int cv_bind(cv_ctx *c, int role, int h)
{
    if (!c || role < 0 || role >= CV_NUM_ROLES) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (h >= 0) {
        MapObj *m = get(c, h);
        if (!m) return -EBADF;
        const HostMap *hm = m->hm.get();
        const bool lpm = hm->is_lpm();
        switch (role) {
        case CV_ROLE_CIDR4_FIX: if (lpm || hm->ks != 8) return -EINVAL; break;
        case CV_ROLE_CIDR6_FIX: if (lpm || hm->ks != 20) return -EINVAL; break;
        case CV_ROLE_CIDR4_DYN: if (!lpm || hm->ks != 8) return -EINVAL; break;
        case CV_ROLE_CIDR6_DYN: if (!lpm || hm->ks != 20) return -EINVAL; break;
        case CV_ROLE_LXC: if (lpm || hm->ks != 20 || hm->vs != 48) return -EINVAL; break;
        case CV_ROLE_IPCACHE: if (!lpm || hm->ks != 24 || hm->vs != 8) return -EINVAL; break;
        case CV_ROLE_LB4_SERVICES: if (lpm || hm->ks != 8 || hm->vs != 12) return -EINVAL; break;
        case CV_ROLE_LB6_SERVICES: if (lpm || hm->ks != 20 || hm->vs != 24) return -EINVAL; break;
        case CV_ROLE_LB4_REVNAT: if (lpm || hm->ks != 2 || hm->vs != 6) return -EINVAL; break;
        case CV_ROLE_LB6_REVNAT: if (lpm || hm->ks != 2 || hm->vs != 18) return -EINVAL; break;
        default: break;
        }
    }
    c->role[role] = h;
    c->role_version[role] = (uint64_t)-1;   // force recompilation
    return 0;
}

int cv_endpoint_add(cv_ctx *c, uint16_t lxc_id, uint32_t seclabel, int policy_map, int ct4_map)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    MapObj *p = policy_map >= 0 ? get(c, policy_map) : nullptr;
    MapObj *t = ct4_map >= 0 ? get(c, ct4_map) : nullptr;
    if ((policy_map >= 0 && !p) || (ct4_map >= 0 && !t)) return -EBADF;
    if (p && (p->hm->ks != 8 || p->hm->vs != 24 || p->hm->is_lpm())) return -EINVAL;
    if (t && (t->hm->ks != 14 || t->hm->vs != 56 || t->hm->is_lpm())) return -EINVAL;
    for (auto &e : c->eps) if (e.lxc_id == lxc_id) return -EEXIST;
    if (c->device >= 0 && set_device(c)) return -ENODEV;   // (host-only: the endpoint table alone)
    if (p && !p->is_policy) { p->is_policy = true; p->pol_version = 0; }
    if (t && t->kind != MK_CT4 && c->device >= 0) {
        int r = compile_ct(c, t);
        if (r) return r;
    }
    c->eps.push_back(Endpoint{lxc_id, seclabel, policy_map, ct4_map});
    c->eps_dirty = true;
    c->eps_gen++;
    return (int)c->eps.size() - 1;
}

int cv_endpoint_config(cv_ctx *c, int ep, const cv_endpoint_cfg *cfg)
{
    if (!c || !cfg) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (ep < 0 || (size_t)ep >= c->eps.size()) return -EINVAL;
    MapObj *t6 = cfg->ct6_map >= 0 ? get(c, cfg->ct6_map) : nullptr;
    if (cfg->ct6_map >= 0 && !t6) return -EBADF;
    if (t6 && (t6->hm->ks != 40 || t6->hm->vs != 56 || t6->hm->is_lpm())) return -EINVAL;
    if (t6 && t6->kind != MK_CT6 && c->device >= 0) {
        if (t6->kind != MK_PLAIN) return -EINVAL;
        if (set_device(c)) return -ENODEV;
        int r = compile_ct6(c, t6);
        if (r) return r;
    }
    Endpoint &e = c->eps[ep];
    e.ct6 = cfg->ct6_map;
    e.ipv4 = cfg->ipv4;
    memcpy(e.ipv6, cfg->ipv6, 16);
    e.mac[0] = rd32(cfg->mac); e.mac[1] = rd16(cfg->mac + 4);
    e.node_mac[0] = rd32(cfg->node_mac); e.node_mac[1] = rd16(cfg->node_mac + 4);
    c->eps_dirty = true;
    c->eps_gen++;
    return 0;
}

int cv_node_config(cv_ctx *c, const cv_node_cfg *cfg)
{
    if (!c || !cfg) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->node = *cfg;
    return 0;
}

// how the agent's writes reached the device so far: stream-ordered publications of
// incremental changes, and table rebuilds (a boundary that waited for the device)
int cv_publish_stats(cv_ctx *c, uint64_t *publications, uint64_t *rebuilds)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (publications) *publications = c->publications;
    if (rebuilds) *rebuilds = c->full_compiles;
    return 0;
}

int cv_sync(cv_ctx *c)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    return sync_locked(c, nullptr);         // (fails with -EPROTO after a walker error: walker_error)
}

int cv_xdp_prefilter(cv_ctx *c, const cv_batch *b, cv_out *o, void *stream)
{
    if (!c) return -EINVAL;
    int r = check_batch(b);
    if (r) return r;
    std::lock_guard<std::mutex> g(c->mu);
    if ((r = set_device(c)) || (r = sync_locked(c, (hipStream_t)stream))) return r;
    StreamScope scope(c, (hipStream_t)stream);
    r = launch_xdp_prefilter(params(c), to_dev(b), to_dev(o), (hipStream_t)stream);
    return r;
}

int cv_policy_ingress(cv_ctx *c, int ep, const cv_batch *b, cv_out *o, void *stream)
{
    if (!c) return -EINVAL;
    int r = check_batch(b);
    if (r) return r;
    std::lock_guard<std::mutex> g(c->mu);
    if (ep < 0 || (size_t)ep >= c->eps.size() || c->eps[ep].policy < 0) return -EINVAL;
    if ((r = set_device(c)) || (r = sync_locked(c, (hipStream_t)stream))) return r;
    StreamScope scope(c, (hipStream_t)stream);
    const DpParams p = params(c);
    const HashTable pol = get(c, c->eps[ep].policy)->pol.view;
    for (uint32_t off = 0; off < b->n && !r; off += c->chunk) {
        const uint32_t n = std::min(c->chunk, b->n - off);
        r = launch_policy_ingress(p, ep, chunk(b, off, n), chunk(o, off), (hipStream_t)stream);
        if (!r) r = launch_policy_fold(pol, (hipStream_t)stream);
    }
    return r;
}

int cv_netdev_ingress(cv_ctx *c, const cv_batch *b, uint32_t now, int with_prefilter, cv_out *o, void *stream)
{
    if (!c) return -EINVAL;
    int r = check_batch(b);
    if (r) return r;
    std::lock_guard<std::mutex> g(c->mu);
    for (auto &e : c->eps) if (e.ct4 < 0 || e.policy < 0) return -EINVAL;
    if ((r = set_device(c)) || (r = sync_locked(c, (hipStream_t)stream))) return r;
    StreamScope scope(c, (hipStream_t)stream);
    const uint32_t cmax = std::min(b->n, c->chunk);
    if ((r = ensure_groups(c, cmax, false))) return r;
    std::set<const void *> seen;
    std::vector<HashTable> pols;
    for (auto &e : c->eps) {
        const HashTable &t = get(c, e.policy)->pol.view;
        if (seen.insert(t.vals).second) pols.push_back(t);
    }
    DpParams p = params(c);
    const std::vector<MapObj *> cts = batch_ct_maps(c);
    for (uint32_t off = 0, n; off < b->n; off += n) {     // sub-batches in packet order
        // a launch whose creates (at most the tuple and its ICMP twin per packet) fit runs
        // at full width; one that may reach a CT map's max_entries runs admitted
        // (run_admitted: any number of CT maps, each map's walk a segment of one scan)
        n = std::min(c->chunk, b->n - off);
        // short of room for 2 n creates: a launch of room / 2 packets (>= 2^20, so it still
        // fills the device) surely fits and runs at full width without the admission passes
        // -- a right-sized table (max_entries near twice the live entries) is always short of
        // 2 n for a 2^24-packet batch, though its real creates are a fraction of that
        uint32_t fit_n = ct_fit_count(c, cts, n, 2);
        if (fit_n < n && fit_n >= std::min<uint32_t>(n, SPLIT_MIN)) n = fit_n;
        bool fits = ct_fits(c, cts, n, 2);
        if (!fits && cts.size() > 1)                      // (many maps: each map's own bound)
            fits = ct_bound_fits(c, p, chunk(b, off, n), nullptr, 0, nullptr, 0, cts, (hipStream_t)stream);
        GroupScratch gs = next_groups(c, 1, (hipStream_t)stream);
        gs.gbits = gbin_bits(n);
        if (!fits) {
            r = run_admitted(c, p, chunk(b, off, n), chunk(o, off, b->stride), now, with_prefilter, gs, cts,
                             (hipStream_t)stream);
        } else {
            r = launch_netdev_ingress(p, chunk(b, off, n), now, with_prefilter, chunk(o, off, b->stride), gs,
                                      (hipStream_t)stream);
        }
        p.ct_guard = 0;
        if (r) return r;
        for (const HashTable &t : pols)
            if ((r = launch_policy_fold(t, (hipStream_t)stream))) return r;
        if (getenv("CV_GROUP_STATS")) group_stats(c, "netdev", (hipStream_t)stream, false);
    }
    return 0;
}

}  // extern "C"

namespace {

// cv_lxc_egress, and with `deliver` its split form (cv_lxc_egress_split)
int lxc_egress(cv_ctx *c, const cv_batch *b, const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash,
               uint32_t now, cv_out *o, uint8_t *deliver, void *stream)
{
    if (!c) return -EINVAL;
    if (deliver && (reinterpret_cast<uintptr_t>(deliver) & 15)) return -EINVAL;
    auto oc = [&](uint32_t off) {
        OutDev d = chunk(o, off, b->stride);
        if (deliver) d.deliver = reinterpret_cast<uint4 *>(deliver) + (size_t)off * DEL_SLOTS;
        return d;
    };
    int r = check_batch(b);
    if (r) return r;
    std::lock_guard<std::mutex> g(c->mu);
    for (auto &e : c->eps) if (e.ct4 < 0 || e.policy < 0) return -EINVAL;
    if ((r = set_device(c)) || (r = sync_locked(c, (hipStream_t)stream))) return r;
    StreamScope scope(c, (hipStream_t)stream);
    const uint32_t cmax = std::min(b->n, c->chunk);
    if ((r = ensure_groups(c, cmax, true))) return r;
    std::set<const void *> seen;
    std::vector<HashTable> pols;
    for (auto &e : c->eps) {
        const HashTable &t = get(c, e.policy)->pol.view;
        if (seen.insert(t.vals).second) pols.push_back(t);
    }
    DpParams p = params(c);
    const std::vector<MapObj *> cts = batch_ct_maps(c);
    const bool guarded = c->hk.egress_guarded;                    // (tests: the planned launches)
    const bool one_map = egress_admissible(cts) && !c->hk.eam_force;   // (measurements: the many-map form)
    for (uint32_t off = 0, n; off < b->n; off += n) {     // sub-batches in packet order
        // a launch whose creates (at most 7 per packet) fit runs at full width; one that may
        // reach max_entries runs admitted: lxc_admitted with one CT map per family,
        // lxc_admitted_maps (windows of EAM_WINDOW packets) with more.  Short of room for
        // 7 n creates, a launch of room / 7 packets (>= 2^20) surely fits and runs without
        // the admission passes.
        n = std::min(c->chunk, b->n - off);
        const uint32_t fit_n = ct_fit_count(c, cts, n, 7);
        if (fit_n < n && fit_n >= std::min<uint32_t>(n, SPLIT_MIN)) n = fit_n;
        bool fits = ct_fits(c, cts, n, 7);
        if (!fits && !one_map && !guarded)                // (many maps: each map's own bound)
            fits = ct_bound_fits(c, p, chunk(b, off, n), nullptr, 1, src_ep ? src_ep + off : nullptr, ep0, cts,
                                 (hipStream_t)stream);
        if (!fits && !one_map && n > EAM_WINDOW) {
            n = EAM_WINDOW;
            fits = ct_fits(c, cts, n, 7);
        }
        if (!fits && guarded) n = ct_plan(c, cts, n, 7, (hipStream_t)stream, &p.ct_guard);
        BatchDev bc = chunk(b, off, n);
        bc.hash = flow_hash ? flow_hash + off : nullptr;             // skb hash of the drop notifications
        if (!fits && !guarded) {
            const uint16_t *se = src_ep ? src_ep + off : nullptr;
            const uint32_t *fh = flow_hash ? flow_hash + off : nullptr;
            const OutDev od = oc(off);
            if (one_map) {
                r = lxc_admitted(c, p, bc, se, ep0, fh, now, od, cts, (hipStream_t)stream);
            } else {
                r = lxc_admitted_maps(c, p, n, se, ep0, cts, (hipStream_t)stream, [&](const DpParams &pp) {
                    GroupScratch gs = next_groups(c, 3, (hipStream_t)stream);
                    gs.gbits = gbin_bits(n);
                    return launch_lxc_egress(pp, bc, se, ep0, fh, now, od, gs, (hipStream_t)stream);
                }, true, "egress");
            }
            // no fixed point (the state is back as before the chunk), or no room for the
            // state's copy (nothing ran): the chunk again in planned launches, one guarded
            // packet at a time next to the limit
            const bool again = r == -EAGAIN || r == -ENOMEM;
            for (uint32_t o2 = off, m; again && o2 < off + n; o2 += m) {
                m = ct_plan(c, cts, off + n - o2, 7, (hipStream_t)stream, &p.ct_guard);
                BatchDev bm = chunk(b, o2, m);
                bm.hash = flow_hash ? flow_hash + o2 : nullptr;
                GroupScratch gs = next_groups(c, 3, (hipStream_t)stream);
                gs.gbits = gbin_bits(m);
                int r2 = launch_lxc_egress(p, bm, src_ep ? src_ep + o2 : nullptr, ep0,
                                           flow_hash ? flow_hash + o2 : nullptr, now, oc(o2), gs,
                                           (hipStream_t)stream);
                p.ct_guard = 0;
                for (const HashTable &t : pols)
                    if (!r2) r2 = launch_policy_fold(t, (hipStream_t)stream);
                if (r2) return r2;
                if (o2 + m == off + n) r = 0;
            }
        } else {
            GroupScratch gs = next_groups(c, 3, (hipStream_t)stream);
            gs.gbits = gbin_bits(n);                              // (the binned grouping of the components)
            r = launch_lxc_egress(p, bc, src_ep ? src_ep + off : nullptr, ep0, flow_hash ? flow_hash + off : nullptr,
                                  now, oc(off), gs, (hipStream_t)stream);
        }
        p.ct_guard = 0;
        if (r) return r;
        for (const HashTable &t : pols)
            if ((r = launch_policy_fold(t, (hipStream_t)stream))) return r;
        if (getenv("CV_GROUP_STATS")) group_stats(c, "egress", (hipStream_t)stream, true);
    }
    return 0;
}

}  // namespace

extern "C" {

int cv_lxc_egress(cv_ctx *c, const cv_batch *b, const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash,
                  uint32_t now, cv_out *o, void *stream)
{
    return lxc_egress(c, b, src_ep, ep0, flow_hash, now, o, nullptr, stream);
}

int cv_lxc_egress_split(cv_ctx *c, const cv_batch *b, const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash,
                        uint32_t now, cv_out *o, uint8_t *deliver, void *stream)
{
    if (!deliver) return -EINVAL;
    return lxc_egress(c, b, src_ep, ep0, flow_hash, now, o, deliver, stream);
}

int cv_lxc_deliver(cv_ctx *c, const uint8_t *records, uint32_t n, int v6, uint32_t now, cv_out *o, void *stream)
{
    if (!c || (n && !records) || (reinterpret_cast<uintptr_t>(records) & 15)) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    for (auto &e : c->eps) if (e.ct4 < 0 || e.policy < 0) return -EINVAL;
    int r;
    if ((r = set_device(c)) || (r = sync_locked(c, (hipStream_t)stream))) return r;
    StreamScope scope(c, (hipStream_t)stream);
    const uint32_t cmax = std::min(n, c->chunk);
    if ((r = ensure_groups(c, std::max<uint32_t>(cmax, 1), true))) return r;   // (gres / gdel_ev: egress scratch)
    std::set<const void *> seen;
    std::vector<HashTable> pols;
    for (auto &e : c->eps) {
        const HashTable &t = get(c, e.policy)->pol.view;
        if (seen.insert(t.vals).second) pols.push_back(t);
    }
    DpParams p = params(c);
    const std::vector<MapObj *> cts = batch_ct_maps(c);
    const bool guarded = c->hk.egress_guarded;
    for (uint32_t off = 0, m; off < n; off += m) {
        // a record creates at most the tuple and its ICMP twin in its destination's map: a
        // launch that surely fits runs whole, else admitted (lxc_admitted_maps with the
        // records' slot-1 budgets, windows of EAM_WINDOW), else planned launches (one
        // guarded record at a time next to the limit)
        m = std::min(c->chunk, n - off);
        bool fits = ct_fits(c, cts, m, 2);
        if (!fits && !guarded) {                          // (many maps: each destination map's own bound)
            const BatchDev bd{nullptr, v6 ? 128u : 64u, m, nullptr, nullptr, off, nullptr};
            fits = ct_bound_fits(c, p, bd, reinterpret_cast<const uint4 *>(records) + (size_t)off * DEL_SLOTS, 2,
                                 nullptr, 0, cts, (hipStream_t)stream);
        }
        if (!fits && m > EAM_WINDOW) {
            m = EAM_WINDOW;
            fits = ct_fits(c, cts, m, 2);
        }
        auto one = [&](uint32_t o2, uint32_t k, const DpParams &pp) {
            GroupScratch gs = next_groups(c, 1, (hipStream_t)stream);
            gs.gbits = gbin_bits(k);
            gs.del = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(records)) + (size_t)o2 * DEL_SLOTS;
            const BatchDev bd{nullptr, v6 ? 128u : 64u, k, nullptr, nullptr, o2, nullptr};
            return launch_lxc_deliver(pp, bd, now, chunk(o, o2), gs, v6, (hipStream_t)stream);
        };
        r = -EAGAIN;
        if (!fits && !guarded)
            r = lxc_admitted_maps(c, p, m, nullptr, 0, cts, (hipStream_t)stream,
                                  [&](const DpParams &pp) { return one(off, m, pp); }, false, "deliver", v6);
        if (fits) r = one(off, m, p);
        for (uint32_t o2 = off, k; (r == -EAGAIN || r == -ENOMEM) && o2 < off + m; o2 += k) {
            k = ct_plan(c, cts, off + m - o2, 2, (hipStream_t)stream, &p.ct_guard);
            int r2 = one(o2, k, p);
            p.ct_guard = 0;
            if (r2) return r2;
            if (o2 + k == off + m) r = 0;
        }
        p.ct_guard = 0;
        if (r) return r;
        for (const HashTable &t : pols)
            if ((r = launch_policy_fold(t, (hipStream_t)stream))) return r;
    }
    return 0;
}

int cv_metrics_read(cv_ctx *c, uint64_t *out)
{
    if (!c || !out) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_device(c)) return -ENODEV;
    (void)hipDeviceSynchronize();
    return hipMemcpy(out, c->metrics, METRICS_WORDS * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -EIO;
}

int cv_metrics_reset(cv_ctx *c)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_device(c)) return -ENODEV;
    return hipMemset(c->metrics, 0, METRICS_WORDS * 8) == hipSuccess ? 0 : -EIO;
}

uint64_t *cv_metrics_device_ptr(cv_ctx *c) { return c ? reinterpret_cast<uint64_t *>(c->metrics) : nullptr; }

// the cilium_events drop stream (DROP_NOTIFY) into caller-owned device buffers
int cv_notify_attach(cv_ctx *c, cv_drop_notify *records, uint32_t capacity, uint32_t *count)
{
    if (!c || (records && !count)) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->device >= 0) (void)hipDeviceSynchronize();
    c->notify = records;
    c->notify_cap = records ? capacity : 0;
    c->notify_count = records ? count : nullptr;
    return 0;
}

// the cilium_events trace stream (TRACE_NOTIFY) into caller-owned device buffers
int cv_trace_attach(cv_ctx *c, cv_trace_notify *records, uint32_t capacity, uint32_t *count, uint32_t aggregation,
                    uint32_t ingress_ifindex)
{
    if (!c || (records && !count)) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->device >= 0) (void)hipDeviceSynchronize();
    c->trace = records;
    c->trace_cap = records ? capacity : 0;
    c->trace_count = records ? count : nullptr;
    c->trace_agg = aggregation;
    c->ingress_ifindex = ingress_ifindex;
    return 0;
}

int cv_metrics_attach(cv_ctx *c, uint64_t *buf)
{
    if (!c) return -EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->metrics = buf ? reinterpret_cast<unsigned long long *>(buf) : c->metrics_own.as<unsigned long long>();
    return 0;
}

}  // extern "C"
