// cv_dp.hpp — the datapath parameter block handed to the gfx950 kernels, and the
// launch entry points implemented in cv_kernels.hip.
#pragma once
#include "cv_hash.hpp"
#include "cv_lpm.hpp"

namespace cv {

// policy side values: 32-B slots {proxy_port u16, pad, packets u64 @8, bytes u64 @16}
// (struct policy_entry); the datapath adds {count:25 | bytes:39} deltas with one atomic
// per hit into HashTable::aux[slot] and k_policy_fold folds them into packets/bytes
// after every launch chunk of at most MAX_CHUNK packets (no field can overflow).
constexpr uint32_t MAX_CHUNK = 1u << 24;

struct EpDev {                 // one endpoint program (bpf_lxc.c), its maps and lxc_config.h constants
    HashTable policy;          // PolicySpec + 32-B side values {proxy_port, pad, packets, bytes}
    HashTable ct4;             // Ct4Spec + 64-B side values (struct ct_entry)
    HashTable ct6;             // Ct6Spec + 64-B side values
    uint32_t seclabel;
    uint32_t lxc_id;           // LXC_ID (EVENT_SOURCE of the program)
    uint32_t ct_id;            // identifies the CT map (group key component)
    uint32_t ipv4;             // LXC_IPV4 (raw network-order word); 0 = no IPv4 programs
    uint32_t ipv6[4];          // LXC_IP
    uint32_t mac[2];           // LXC_MAC bytes 0-3 | 4-5
    uint32_t node_mac[2];      // NODE_MAC
};

// The fields the conntrack stages read per packet, in one 64-B line per endpoint (policy
// and CT tables; value strides are fixed: 32-B policy_entry slots, 32-B ct_entry side
// slots), so a lane reads one line instead of the table structs' fields scattered over
// EpDev.  Two arrays: the CT4 map's (IPv4 stages) and the CT6 map's (IPv6 stages).
struct EpHot {
    uint32_t *pol_buckets;
    uint8_t *pol_vals;
    unsigned long long *pol_aux;
    uint32_t *ct_buckets;
    uint8_t *ct_vals;
    unsigned long long *ct_live;
    uint32_t pol_mask, ct_mask;    // bucket counts - 1 (< 2^32)
    uint32_t seclabel;             // SECLABEL
    uint32_t ct_v4;                // ct_id & EPH_CT_ID (the CT4 map's group-key salt) | EPH_V4 (LXC_IPV4 set)
};
static_assert(sizeof(EpHot) == 64, "one line per endpoint");
constexpr uint32_t EPH_CT_ID = 0x3FFFFFFFu, EPH_V4 = 0x80000000u;

// Copy-on-first-write of conntrack slots (egress admission with many CT maps, cv_ctx.cpp
// lxc_admitted_maps): before a pass's first write to a CT slot, the slot as it was -- its
// tag byte, key and hot words, side slot -- goes to a log; a pass that was not the
// sequential run is undone from the log (k_snap_restore) instead of from a copy of every
// map.  "First" is the slot's bit in its bucket's spare word (the bucket line the write
// touches anyway: CT4 buckets hold 30 of their 32 words, CT6 62 of 64), set with one
// atomic OR and cleared from the log after every pass (k_snap_clear).  The log has
// SNAP_PER entries per packet, written by the packet's own stages in order (no
// allocation atomics).
struct Snap {
    uint4 *log;                // per entry SNAP_U4 x 16 B: {bucket address, s | tag << 8 | KS << 16 | spare
                               // word << 24, the slot's KS bucket words from KEY0 at word 4, the side slot's
                               // 8 words at word 24, the side slot's address at word 32}
    uint8_t *cnt;              // per packet the entries written
    uint32_t n;                // packets
    uint32_t pad;
    uint32_t *err;             // set when a packet has more entries than SNAP_PER (the pass cannot be undone:
                               // loud failure)
};
constexpr uint32_t SNAP_U4 = 9, SNAP_PER = 8;

struct DpParams {              // by value as the kernel argument
    uint32_t flags;
    uint32_t n_eps;
    HashTable cidr4_fix, cidr6_fix, lxc4, lxc6;
    Lpm4 cidr4_dyn, ipc4;
    Lpm6 cidr6_dyn, ipc6;
    const EpDev *eps;
    const EpHot *ephot;        // per endpoint, same index as eps (CT4 map)
    const EpHot *ephot6;       // the same with the endpoint's CT6 map
    const uint16_t *ep_of_lxc; // lxc_id -> endpoint index + 1 (0 = no program)
    unsigned long long *metrics;   // [256][4][2]
    // load balancer (lb.h): services and dense reverse-NAT tables indexed by the raw u16 key
    HashTable lb4, lb6;        // Lb4Spec / Lb6Spec
    const uint32_t *revnat4;   // [65536][2]  {address, port | valid << 16}
    const uint32_t *revnat6;   // [65536][8]  {address[4], port | valid << 16, 0, 0, 0}
    // node_config.h constants (raw network-order words)
    uint32_t v4_cluster_mask, v4_cluster_range, v4_loopback;
    uint32_t router6[4];
    uint32_t host_mac[2];      // HOST_IFINDEX_MAC bytes 0-3 | 4-5
    uint32_t net_mac[2];       // CILIUM_NET_MAC (rewrite_dmac_to_host, bpf_netdev.c:156-169)
    // drop notifications (cv_notify_attach): cv_drop_notify records of 10 words
    uint32_t *notify;
    uint32_t notify_cap;
    uint32_t *notify_count;
    // trace notifications (cv_trace_attach): cv_trace_notify records of 10 words
    uint32_t *trace;
    uint32_t trace_cap;
    uint32_t *trace_count;
    uint32_t trace_agg;        // MONITOR_AGGREGATION
    uint32_t ingress_ifindex;  // skb->ingress_ifindex of from_netdev
    uint32_t ct_guard;         // 1: creates check the CT map's live count against max_entries (cv_ctx.cpp admission)
    uint32_t win_lo, win_span; // the conntrack stages run the packets in [win_lo, win_lo + win_span) (admission
                               // windows; 0, ~0 otherwise)
    const uint8_t *budget;     // admission: per packet the creates of new CT entries that succeed, or null
    // egress admission (cv_ctx.cpp lxc_admitted): per packet the budget left for its next
    // stage, and its intent {creates tried (3 bits), deletes << 3, CT map (0 CT4, 1 CT6) << 4}
    uint8_t *eg_left;
    uint8_t *eg_intent;
    // many CT maps (lxc_admitted_maps): the local delivery's creates and delete go to the
    // destination's map, with a budget and an intent of their own ({tried, deletes << 3}),
    // and its endpoint; null with one map per family (one budget per packet)
    uint8_t *eg_left2;
    uint8_t *eg_intent2;
    uint16_t *eg_dst;
    const Snap *snap;          // in device memory (not the kernel argument: its address would copy the
                               // parameters to scratch); null: off
    // every endpoint on one policy map and one CT4 map with LXC_IPV4 set (cv_ctx.cpp): the
    // netdev stages take that line from here instead of a per-packet EpHot read
    uint32_t uni4_on, uni6_on;
    EpHot uni4, uni6;          // (uni6: one policy and CT6 map for every endpoint)
};

// Exact conntrack admission next to max_entries (cv_kernels.hip "conntrack
// admission", cv_ctx.cpp run_admitted), for any number of CT maps: every endpoint's
// CT4 / CT6 map has an index in the launch's map list (per-endpoint maps:
// ConntrackLocal), and each map's walk is one segment of a scan over the packets with
// creates or deletes sorted by (map, packet).  (Launch chunks hold <= MAX_CHUNK = 2^24 packets.)
constexpr uint32_t ADMIT_NO_MAP = 0xFFFFu;  // (an endpoint without a CT map of that family)
struct Admit {
    const uint16_t *ep_mi4, *ep_mi6;   // per endpoint: its CT4 / CT6 map's index in the map list
    unsigned long long *const *live;   // per map: its live-entry count
    const unsigned long long *cap;     // per map: max_entries
    uint32_t nmaps;
    uint32_t lo;                       // the first packet not yet run
    uint32_t pass;                     // the pass over this window (0: every packet from lo)
    uint8_t *ib;                       // per packet: creates A | deletes D << 2 | read a budget << 5 |
                                       // unsure << 6 (bit 7: too many changed keys in its run)
    uint16_t *mi;                      // per packet: its CT map's index (k_ct_intent)
    uint8_t *budget;                   // per packet: how many of its creates of new entries succeed (the
                                       // previous pass's: what k_ct_intent assumes of earlier creates)
    unsigned long long *keys;          // map << 24 | packet of every packet from lo with creates or deletes
                                       // (hi[4] of them, sorted into keys_sorted: the walks' elements)
    unsigned long long *keys_sorted;
    uint32_t *tsum;                    // per scan tile of keys_sorted: the segmented (sum, prefix minimum)
    uint32_t *hi;                      // [0] the first unsure packet (the window's end), [1] the first
                                       // packet whose intent changed from the previous pass, [2] the first
                                       // packet whose intent rests on an earlier member's budget, [3] error
                                       // bits (ADMIT_ERR_*: the host fails the batch with -EPROTO), [4] the
                                       // walks' elements (k_adm_keys)
    uint32_t inject;                   // test hook (CV_ADMIT_INJECT): this packet's map index is corrupted
                                       // after the intents (~0u: none)
    void *sort_tmp;                    // radix-sort scratch
    size_t sort_bytes;
    unsigned long long *evt;           // k_ct_intent's spill tables: 4 slots of 16 B per `order` word
    uint32_t stamp;                    // this pass's (spill-table slots of other passes are free)
};
// a packet's endpoint has no CT map in the list (k_ct_intent), a packet's map index is
// past nmaps (k_adm_keys): a stale or corrupt intent, failed loudly instead of indexing
// past the map arrays
enum : uint32_t { ADMIT_ERR_MAP = 1, ADMIT_ERR_IB = 2 };
// the 64-bit key sort of the admission walks (cv_sort.hip, rocPRIM radix sort over the
// low end_bit bits); tmp = null: *bytes = the scratch size n keys need
int sort_keys64(void *tmp, size_t *bytes, const unsigned long long *in, unsigned long long *out, uint32_t n,
                int end_bit, hipStream_t s);

// Exact egress admission (cv_kernels.hip "egress admission", cv_ctx.cpp lxc_admitted):
// whether a pass was the sequential run, and the next pass's budgets (one CT4, one CT6 map)
struct EAdmit {
    const uint8_t *intent;             // per packet (DpParams::eg_intent)
    const uint8_t *used;               // the budgets the pass ran with
    uint8_t *next;                     // the next pass's budgets
    uint32_t *tsum;                    // per map and scan tile: (sum, prefix minimum)
    const unsigned long long *live0[2];  // the maps' live counts as the window started
    unsigned long long cap[2];         // max_entries (CT4, CT6)
    uint32_t *flag;                    // set when a packet's creates differ from the sequential run's
    uint32_t n;
};

// Exact egress admission with any number of CT maps (lxc_admitted_maps): a packet's
// elements are its source program's creates and deletes (slot 0, the source endpoint's
// map) and its local delivery's (slot 1, the destination's map), keyed map << 25 |
// packet << 1 | slot and sorted, each map's walk one segment of the (sum, prefix
// minimum) scan; the check and the next budgets per element as EAdmit's per packet
struct EAdmitM {
    const uint8_t *intent, *intent2;   // per packet (DpParams::eg_intent / eg_intent2)
    const uint8_t *used, *used2;       // the budgets the pass ran with
    uint8_t *next, *next2;             // the next pass's budgets
    const uint16_t *src_ep;            // per packet the source endpoint, or null: ep0
    uint32_t ep0;
    const uint16_t *dst_ep;            // per packet the delivery's endpoint (DpParams::eg_dst)
    const uint16_t *ep_mi4, *ep_mi6;   // per endpoint its CT4 / CT6 map's index (ADMIT_NO_MAP: none)
    uint32_t n_eps;
    const unsigned long long *live0;   // per map its live count as the window started
    const unsigned long long *cap;     // per map max_entries
    unsigned long long *keys, *keys_sorted;
    void *sort_tmp;
    size_t sort_bytes;
    uint32_t *tsum;
    uint32_t *cnt;                     // [0] elements, [1] elements not as in the sequential run, [2] a bad
                                       // map index, [3] the first packet of such an element
    uint32_t n, nmaps;
};
int launch_eam_first(const EAdmitM &a, hipStream_t s);     // first-pass budgets: 0 in a full source map, else 7
int launch_eam_keys(const EAdmitM &a, hipStream_t s);      // the elements -> keys, cnt[0] their number
int launch_eam_walks(const EAdmitM &a, uint32_t K, hipStream_t s);   // sort + scan: cnt[1], next budgets
int launch_snap_restore(const Snap &sn, hipStream_t s);
int launch_snap_clear(const Snap &sn, hipStream_t s);   // every pass: the spare-word bits of the logged slots
int launch_scatter_u64(unsigned long long *const *ptrs, const unsigned long long *in, uint32_t n, hipStream_t s);

struct BatchDev {
    const uint8_t *frames;
    uint32_t stride, n;
    const uint32_t *len;
    const uint32_t *mark;
    uint32_t base;             // index of packet 0 in the caller's batch (launch chunks)
    const uint32_t *hash;      // per-packet skb hash (cv_lxc_egress flow_hash) or null
};

struct OutDev {
    uint8_t *xdp;
    int32_t *ret;
    uint32_t *identity;
    uint8_t *ct;
    uint16_t *proxy;
    uint8_t *nl, *nu;          // optional accounting of map lookups / entry writes
    int32_t *reason;           // DROP_* behind a TC_ACT_SHOT, else 0
    uint8_t *frames;           // optional output records (the batch's stride), see cv_out.frames_out
    uint4 *deliver;            // egress split (cv_lxc_egress_split): a packet delivered to a local endpoint
                               // leaves its 64-B delivery record here (DEL_SLOTS x 16 B) with ret E_DEFER
                               // instead of running the destination's program, or null
};

struct GroupScratch {          // address-pair grouping for conntrack (config 3)
    unsigned long long *table; // 2 * cap u64: {epoch << 32 | hash, epoch << 32 | head}
    uint32_t cap_mask;
    uint32_t epoch;
    uint32_t *gslot;           // per packet: group slot or ~0
    uint32_t *next;            // per packet: previous inserter in the group or ~0
    uint4 *srec;               // per packet 2 x 16 B (netdev path, packets handed to the policy
                               // program): [0] the IPv4 stage record (skb4_pack), [1] {the
                               // packed protocol word, access bits | nl << 16 | nu << 24,
                               // meta = ep index | skip_proxy << 16 | ifindex != 0 << 17,
                               // the source label}
    unsigned long long *parent;// per table slot: epoch << 32 | union-find parent (egress path)
    uint32_t *eg;              // per packet: EG_WORDS words of egress scratch (egress path)
    uint32_t serial;           // launch serial (never reset; tags deferred CT writes)
    uint32_t *order;           // 2 words per packet: the runs {size, members} of the binned grouping
    uint32_t *cursor;          // [CURSOR_WORDS] zeroed per launch: [0..2] cursors into `order`,
                               // [qctr(q, k)] length of sub-queue k of queue q (one 128-B line each)
    uint32_t *queue;           // dense lists of group slots (one lane per group), QSPLIT regions
    uint32_t qregion;          // words per region
    uint32_t *work;            // per group: `order` offset of its run, in size-class order
    uint32_t *ifx;             // per packet: the destination endpoint's ifindex (netdev path)
    uint32_t *single;          // the packets of singleton groups, dense (k_gbin_group ->
                               // k_heads_place; cursor[SINGLE_WORD0 + q] of them)
    // netdev path (k_gkey_hist / k_gkey_scatter / k_gbin_group): groups by binning
    unsigned long long *pkey;  // per packet: the address-pair key of a staged packet, 0 if none
    uint2 *gent;               // staged packets binned by key: {packet, key low word}
    uint32_t *gcnt;            // per (bin, count block) counts, scanned into offsets in place;
                               // [nbins * GBLK] = the staged total
    unsigned long long *gbig;  // sort space of bins too large for LDS: 2 words per packet
    uint32_t gbits;            // log2 of the number of bins
    uint32_t *single6;         // the singleton packets of the IPv6 queue (Q_NETDEV6)
    uint32_t *work6;           // the IPv6 queue's schedule (`work` of Q_NETDEV6)
    uint32_t *hword;           // per packet: 0, or for a group's first packet (1 + its list) << 26 | its run's
                               // offset in `order` (k_gbin_group -> k_heads_place)
    uint32_t *hcnt;            // per (list, tile) head counts -> positions (k_heads_count / place)
    uint32_t q4;               // the IPv4 queue the binned grouping fills (Q_NETDEV, or Q_LB4 / Q_CT4 on egress)
    uint32_t flat;             // 1: position lists (egress): list t < NPOS - 1 holds member t of every
                               // group, lists NPOS - 1 .. 15 (by size class) the runs of groups past
                               // NPOS - 1 members, in
                               // packet order (k_gbin_group -> k_heads_place)
    uint32_t pos;              // egress: the member position of the current launch pair
    uint4 *res;                // egress: per packet the packed final outputs of the scattered stages
                               // (eg_done), written out in packet order by k_out_unpack
    uint4 *del_ev;             // egress: per packet 2 x 16 B, the event-only part of a delivery record
    uint4 *del;                // egress: per packet DEL_SLOTS x 16 B, the local-delivery record
                               // k_egress_ct hands to k_egress_deliver (listed in `single`)
    uint4 *est;                // egress: per packet 64 B, the conntrack stage's packed input state
                               // (k_egress_pairs -> k_egress_ct)
    uint32_t q6;               // the IPv6 queue the binned grouping fills (Q_NETDEV6, or Q_LB6 / Q_CT6)
    uint32_t *sjob;            // the binned grouping's split keys (elephant address pairs): SJOB_WORDS per
                               // job, ordered tile by tile in parallel by k_gbin_tiles; cursor[SJOB_WORD]
                               // counts them
    uint32_t sjob_cap;         // jobs sjob holds
    uint32_t *hot;             // elephants in parallel (cv_kernels.hip k_hpar_*): per hot run and chunk
    uint32_t hot_chunks;       // chunks it holds
    uint32_t lim;              // packets of this launch (set by the launchers): every list word the
                               // walkers read is a packet < lim or an `order` offset < 2 * lim
    uint32_t *err;             // host-mapped error word of the context: a walker that reads a list
                               // word past the launch stores GERR_* here and skips it (the host fails
                               // its next call with -EPROTO), or null
    uint32_t *gbx;             // the binned grouping's big bins (k_gbig_*): per bin its record + 1 (0:
                               // none), then BIGW words per record (BIG_*)
    uint32_t gbx_cap;          // records gbx holds
};
enum : uint32_t { GERR_INDEX = 1 };
// binning blocks of k_gkey_hist / k_gkey_scatter (each a contiguous packet range), and
// the most bins (2^gbits) a launch uses
constexpr uint32_t GBLK = 256, GBIN_MAX = 1u << 14;
// GroupScratch queues: appends go to one of QSPLIT sub-queues by block index (less
// contention on one counter); blocks b with b % QSPLIT == k hold at most
// n / QSPLIT + BLOCK + QSPLIT packets (grids are multiples of QSPLIT or one block per 256
// packets), so a region of n / QSPLIT + 512 words never overflows.
// Queues filled at the same time (the v4 and v6 lists of one stage) live in different
// banks of `queue`: QSPLIT regions of qregion words each per bank.
enum : int { Q_NETDEV = 0, Q_LB4 = 1, Q_LB6 = 2, Q_CT4 = 3, Q_CT6 = 4, Q_NAT = 5, NQUEUES = 6 };
// the netdev path's IPv6 groups (handle_ipv6 -> ipv6_policy) use the CT6 queue, which the
// egress path alone fills otherwise; it sits in the other bank from Q_NETDEV
constexpr int Q_NETDEV6 = Q_CT6;
// Size-sorted runs (k_heads_place): per queue NCLASS group-size classes, each a count on
// its own line after the sub-queue counters.
constexpr int QSPLIT = 16, QBANKS = 2, NCLASS = 16;
constexpr int CLS0 = 32 + NQUEUES * QSPLIT * 32, CURSOR_WORDS = CLS0 + NQUEUES * NCLASS * 32;
__host__ __device__ constexpr int qbank(int q) { return (q == Q_LB6 || q == Q_CT6) ? 1 : 0; }
__host__ __device__ constexpr int qctr(int q, int k) { return 32 + (q * QSPLIT + k) * 32; }
__host__ __device__ constexpr int qcls(int q, int c) { return CLS0 + (q * NCLASS + c) * 32; }
constexpr int GMAX_WORD0 = 8;   // cursor[8 + q]: the largest group of queue q (diagnostics)
constexpr uint32_t SINGLE_RUN = 0x80000000u; // a list word naming a singleton's packet (diagnostics)
constexpr int SINGLE_WORD0 = 16; // cursor[16 + q]: singleton groups of queue q listed in `single`
constexpr int SJOB_WORD = 24;    // cursor[24]: split-key jobs of the binned grouping (GroupScratch::sjob)
constexpr int BIG_WORD = 25;     // cursor[25]: big-bin records of the binned grouping (GroupScratch::gbx)
// a big bin (>= BIG_MIN entries): a record of BIGW words {bin, key, start, entries, the key's
// members, the other entries, its job (~0: not taken out), the others' fill, per scatter
// tile the key's members [GBLK] (then the tile's fill cursor [GBLK])}
#ifndef CV_BIG_MIN
#define CV_BIG_MIN 2048
#endif
constexpr uint32_t BIG_MIN = CV_BIG_MIN, BIG_PCNT = 8, BIG_FILL = 8 + 256, BIGW = 8 + 512;
// a split-key job: {key, members c, order offset, listed, member base in gbig (u32 words), tile, pad[2],
// head[NPOS <= 8], per tile its member count [GBLK] and offset [GBLK]}
constexpr uint32_t SJOB_HEAD = 8, SJOB_PCNT = 16, SJOB_WORDS = 16 + 2 * 256;
constexpr int EG_WORDS = 16;
// position lists of the egress conntrack stage: one launch per member position, the last
// one continuing the groups past NPOS - 1 members (<= 16: the lists are k_heads' 16).  With
// the continuation on lists by size class, 2 positions beat 3 and 4 (A/B on one box, per
// step: 13.34 / 13.65 / 13.50 ms; round 4, one continuation list: 3 best)
#ifndef CV_NPOS
#define CV_NPOS 2
#endif
constexpr uint32_t NPOS = CV_NPOS;
constexpr uint32_t DEL_SLOTS = 4;                 // (64 B: one aligned half line per record)
// the local-delivery list counter of a position (the netdev queue's sub-queue counters,
// which the egress path does not use)
__host__ __device__ constexpr int del_ctr(bool v6, uint32_t pos) { return 32 + (int)((v6 ? 8u : 0u) + pos) * 32; }

// the binned grouping of the packets whose g.pkey is set (cv_kernels.hip): runs, and the
// lists of the groups' first packets (g.flat: one per queue)
void launch_gbin_groups(const GroupScratch &g, uint32_t n, hipStream_t s);
int launch_policy_fold(const HashTable &pol, hipStream_t s);
int launch_xdp_prefilter(const DpParams &p, const BatchDev &b, const OutDev &o, hipStream_t s);
int launch_policy_ingress(const DpParams &p, int ep, const BatchDev &b, const OutDev &o, hipStream_t s);
int launch_netdev_ingress(const DpParams &p, const BatchDev &b, uint32_t now, int with_prefilter,
                          const OutDev &o, const GroupScratch &g, hipStream_t s);
// the same in parts: front + grouping + schedules, then (per admission window) the
// conntrack stages and the commit of deferred creates
int launch_netdev_front(const DpParams &p, const BatchDev &b, int with_prefilter, const OutDev &o,
                        const GroupScratch &g, hipStream_t s);
int launch_netdev_stages(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o, const GroupScratch &g,
                         hipStream_t s);
// admission, per window from packet a.lo (after launch_netdev_front): every later
// packet's creates and deletes, the window's end (*a.hi) and the budgets
int launch_admission(const DpParams &p, const BatchDev &b, const GroupScratch &g, const Admit &a, hipStream_t s);
// then, with K = a.hi[4] (the packets with creates or deletes), the per-map walks: budgets
int launch_admission_walks(const BatchDev &b, const Admit &a, uint32_t K, hipStream_t s);
int launch_egress_admission(const EAdmit &a, hipStream_t s);
// the destination's policy program of delivery records (cv_lxc_deliver): records in
// g.del, grouped by (destination CT map, address pair), each group in record order
int launch_lxc_deliver(const DpParams &p, const BatchDev &b, uint32_t now, const OutDev &o, GroupScratch g,
                       int v6, hipStream_t s);
// config 5: from-container of the packets' source endpoints (src_ep[i], or ep0)
int launch_lxc_egress(const DpParams &p, const BatchDev &b, const uint16_t *src_ep, uint32_t ep0,
                      const uint32_t *flow_hash, uint32_t now, const OutDev &o, GroupScratch g, hipStream_t s);
// Room check of a launch over many CT maps (ConntrackLocal: every endpoint its own CT4 /
// CT6 map).  A map can only take creates from the packets whose source program or local
// delivery is its endpoint's, so per map a bound of the launch's creates -- w_src per
// packet from the endpoint (egress), w_dst per packet that may be delivered to it: the
// endpoint owning the destination address, or backing a service the packet may be
// served by -- against its room tells whether the launch surely fits every map (then
// it runs at full width, no admission passes).  Packets whose destination the check
// cannot see (an IPv6 extension header it does not walk) count against every map.
struct CtBound {
    unsigned long long *bound;         // per map: creates the launch may make in it
    uint32_t *svc4, *svc6;             // per LB table slot: packets a service master may serve
    uint32_t *flag;                    // [0] some map may fill, [1] packets of unseen destination
    unsigned long long *const *live;   // per map: its live count (map_table)
    const unsigned long long *cap;     // per map: max_entries
    const uint16_t *epmi4, *epmi6;     // per endpoint: its CT4 / CT6 map's index
    const uint16_t *src_ep;            // egress: per packet its source endpoint, or null (ep0)
    uint32_t ep0, nmaps, n_eps;
    uint32_t w_src, w_dst;             // creates per packet in its source's / destination's map
    uint32_t mode;                     // 0 netdev, 1 egress (source + destination), 2 delivery records
};
int launch_ct_bound(const DpParams &p, const BatchDev &b, const uint4 *records, const CtBound &bd, hipStream_t s);

// one run of words the agent's writes changed in a device table (cv_ctx.cpp PatchQueue)
struct PatchRec {
    unsigned long long dst;    // device address of the first word
    uint32_t words, src;       // run length, offset in the staged word array
};
// k_patch: copy every run from the staged words (recs then words, in one device buffer)
int launch_patches(const PatchRec *recs, uint32_t n, const uint32_t *words, hipStream_t s);
// single-element operations on a device-resident conntrack table (map API path):
// op 0 lookup, 1 update (BPF_ANY/NOEXIST/EXIST in flags), 2 delete; v6 selects the
// ipv6_ct_tuple table.  io = {key[KW words], value[16 words], rc}
int launch_ct_op(const HashTable &t, int v6, int op, uint64_t flags, uint32_t *io_dev, hipStream_t s);
// ctmap.GC (GCFilterByTime): mark entries with lifetime < time dead; adds the count
int launch_ct_gc(const HashTable &t, int v6, uint64_t nb, uint32_t time, uint32_t *deleted, hipStream_t s);
int launch_ct_tags(const HashTable &t, int v6, uint64_t nb, unsigned long long *out, hipStream_t s);
// out[k] = *ptrs[k] (the CT maps' live counts in one read)
int launch_gather_u64(unsigned long long *const *ptrs, unsigned long long *out, uint32_t n, hipStream_t s);
// every live entry: slot index (may be null), key words, 16 value words
int launch_ct_scan(const HashTable &t, int v6, uint64_t nb, uint64_t *out_slots, uint32_t *out_keys, uint32_t *out_vals,
                   uint32_t *count, uint32_t max, hipStream_t s);
// parallel initial fill of an empty CT table with n distinct keys
int launch_ct_load(const HashTable &t, int v6, const uint32_t *keys, const uint32_t *vals, uint64_t n, uint32_t *fail,
                   hipStream_t s);

}  // namespace cv
