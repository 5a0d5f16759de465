/*
 * cilium_hip.h — C-ABI of the MI355X batch packet-verdict engine.
 *
 * This is the drop-in boundary for Cilium's L3/L4 verdict path.  It replaces two
 * boundaries of the reference (Taeung/cilium v1.1.90):
 *
 *  (1) the control boundary agent -> tables: the bpf(2) map syscalls wrapped by
 *      pkg/bpf (CreateMap bpf.go:101-139, UpdateElement :146-167, LookupElement
 *      :170-189, DeleteElement :191-216, GetNextKey :218-245, ObjClose :285-297)
 *      that pkg/maps/{cidrmap,ipcache,policymap,ctmap,lbmap,lxcmap,metricsmap}
 *      call.  Keys and values keep the BPF byte layouts of bpf/lib/common.h,
 *      bpf/lib/maps.h and bpf/lib/xdp.h; return codes are the kernel's negative
 *      errnos (-EEXIST, -ENOENT, -E2BIG, -ENOSPC, -EINVAL).
 *
 *  (2) the packet boundary kernel -> program: xdp_start (bpf/bpf_xdp.c:180-184),
 *      from_netdev (bpf/bpf_netdev.c:470-524) and the per-endpoint handle_policy
 *      tail-call target (bpf/bpf_lxc.c:1003-1038), here as batch entry points
 *      over packed frame records in device memory.  Per-packet results use the
 *      reference's own codes (XDP_*, TC_ACT_*, DROP_* of bpf/lib/common.h:237-269).
 *
 * Which map a program reads (the bpf_elf_map names compiled into the reference's
 * programs, and the cilium_policy prog array) becomes an explicit binding:
 * cv_bind() and cv_endpoint_add().  Writes become visible to the datapath at the
 * next batch boundary (cv_sync(), called implicitly by every batch entry point),
 * the way the kernel gives RCU visibility per element.
 *
 * Ownership: the caller owns every key/value/batch buffer; the library owns the
 * device-resident tables.  Errors are negative errnos; nothing aborts.
 * Pointers in cv_batch / cv_out are DEVICE pointers (HBM); `stream` is a
 * hipStream_t (NULL = default stream).
 */
#ifndef CILIUM_HIP_H
#define CILIUM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cv_ctx cv_ctx;

/* ---- BPF map types and update flags (include/linux/bpf.h) ---- */
#define CV_MAP_HASH         1
#define CV_MAP_ARRAY        2
#define CV_MAP_PERCPU_HASH  5
#define CV_MAP_LRU_HASH     9
#define CV_MAP_LPM_TRIE    11
#define CV_ANY      0
#define CV_NOEXIST  1
#define CV_EXIST    2

/* ---- roles: the maps the programs of the reference refer to by name ---- */
#define CV_ROLE_CIDR4_FIX   0   /* v4_fix  HASH lpm_v4_key->lpm_val   (bpf_xdp.c:45-52)  */
#define CV_ROLE_CIDR4_DYN   1   /* v4_dyn  LPM  lpm_v4_key->lpm_val   (bpf_xdp.c:55-62)  */
#define CV_ROLE_CIDR6_FIX   2   /* v6_fix  HASH lpm_v6_key->lpm_val   (bpf_xdp.c:67-74)  */
#define CV_ROLE_CIDR6_DYN   3   /* v6_dyn  LPM  lpm_v6_key->lpm_val   (bpf_xdp.c:77-84)  */
#define CV_ROLE_LXC         4   /* cilium_lxc endpoint_key->endpoint_info (maps.h:27-33) */
#define CV_ROLE_IPCACHE     5   /* cilium_ipcache ipcache_key->remote_endpoint_info (maps.h:151-158) */
#define CV_ROLE_LB4_SERVICES 6  /* cilium_lb4_services lb4_key->lb4_service (lb.h:75-81) */
#define CV_ROLE_LB6_SERVICES 7  /* cilium_lb6_services lb6_key->lb6_service (lb.h:43-49) */
#define CV_ROLE_LB4_REVNAT  8   /* cilium_lb4_reverse_nat u16->lb4_reverse_nat (lb.h:67-73) */
#define CV_ROLE_LB6_REVNAT  9   /* cilium_lb6_reverse_nat u16->lb6_reverse_nat (lb.h:38-44) */
#define CV_NUM_ROLES        10

/* ---- datapath options (compile-time #defines of the reference) ---- */
#define CV_F_FROM_HOST       0x1   /* netdev_config.h FROM_HOST                     */
#define CV_F_HAVE_L4_POLICY  0x2   /* HAVE_L4_POLICY                                */
#define CV_F_DROP_ALL        0x4   /* DROP_ALL (pkg/endpoint/bpf.go)                */
#define CV_F_CT_ACCOUNTING   0x8   /* CONNTRACK_ACCOUNTING (daemon/main.go:676)     */
#define CV_F_POLICY_INGRESS  0x10  /* POLICY_INGRESS                                */
#define CV_F_POLICY_EGRESS   0x20  /* POLICY_EGRESS                                 */
#define CV_F_DEFAULT         0x3b
/* measurement: cv_out.nl / nu count every conntrack lookup / write 32 and every other
 * map lookup / write 1 (the HBM-resident share of the algorithmic bytes) */
#define CV_F_ACCT_SPLIT      0x40

/* ---- per-packet codes (bpf/include/linux/bpf.h:623-628, bpf/include/bpf/api.h:18-25) */
#define CV_XDP_DROP 1
#define CV_XDP_PASS 2
#define CV_TC_ACT_OK 0
#define CV_TC_ACT_SHOT 2
#define CV_TC_ACT_REDIRECT 7
#define CV_E_TRUNC (-1)      /* a header byte the path reads lies beyond the record */
#define CV_E_PUNT  (-2)      /* left the path through a tail call into a responder program
                                (ARP, ICMPv6 NS / echo to the router, hop limit exceeded) */
#define CV_CT_NONE 0xff

/* ---- context ----
 * cv_open(-1, ..) gives a host-only context: the map store and bindings work
 * (agent-side control plane, CPU tests), batch entry points return -ENODEV. */
int  cv_open(int hip_device, cv_ctx **out);
void cv_close(cv_ctx *ctx);
int  cv_set_flags(cv_ctx *ctx, uint32_t flags);
const char *cv_version(void);

/* ---- maps (pkg/bpf/bpf.go:101-297 semantics) ---- */
int cv_map_create(cv_ctx *ctx, int type, uint32_t key_size, uint32_t val_size,
                  uint32_t max_entries, uint32_t flags, int *handle);
int cv_map_update(cv_ctx *ctx, int h, const void *key, const void *val, uint64_t flags);
int cv_map_lookup(cv_ctx *ctx, int h, const void *key, void *val);
int cv_map_delete(cv_ctx *ctx, int h, const void *key);
/* GetNextKey: the element after `key` in the map's walk order, the first when key is
 * NULL or absent, -ENOENT at the end.  O(1) per call (a device CT map walks a snapshot
 * taken once per table generation, in slot order). */
int cv_map_get_next_key(cv_ctx *ctx, int h, const void *key, void *next_key);
int cv_map_close(cv_ctx *ctx, int h);
/* bulk form of cv_map_update in array order (later writes of a key win);
 * *done = elements applied before the first error */
int cv_map_update_batch(cv_ctx *ctx, int h, const void *keys, const void *vals, uint32_t n,
                        uint64_t flags, uint32_t *done);
int cv_map_count(cv_ctx *ctx, int h, uint32_t *count);
/* every entry (keys/vals host buffers of max rows); order unspecified, like a
 * GetNextKey walk.  Returns the number of rows written or -errno. */
int cv_map_dump(cv_ctx *ctx, int h, void *keys, void *vals, uint32_t max);
/* conntrack garbage collection: delete every entry of CT map h (ipv4_ct_tuple or
 * ipv6_ct_tuple keys, ct_entry values) whose lifetime < time; *deleted = count.
 * Replaces ctmap.GC(m, name, GCFilterByTime) / doGC4 / doGC6 and, with
 * time = 0xFFFFFFFF, ctmap.Flush (pkg/maps/ctmap/ctmap.go:247-448).  Runs on the GPU
 * for a bound CT map after waiting for every batch already submitted, on any stream
 * (as every map operation on a device-resident table does).
 *
 * Conntrack capacity: a CT map holds at most max_entries entries.  The reference's
 * CT maps are LRU_HASH (bpf_lxc.c:53-75), which evict at capacity in an order the
 * kernel's per-CPU LRU lists decide; that order is not reproducible, so here a CT map
 * behaves like a kernel HASH map: a create past max_entries fails (-E2BIG, the
 * datapath's DROP_CT_CREATE_FAILED), identically in the oracle.  Size max_entries for
 * the flows the node keeps (HBM: ~137 B per entry at the 60 % bucket load) and run
 * cv_ct_gc.  A batch next to the limit runs at full width with exact admission:
 * from-netdev, every packet's creates and deletes are resolved against its map's room
 * in packet order first; from-container (egress), the pipeline runs with per-packet
 * create budgets and a scan checks them against the sequential run, re-running the
 * launch from a saved state until they agree.  Any number of CT maps
 * (ConntrackLocal: every endpoint its own CT4 / CT6 map) is admitted the same way: each
 * map's walk is a segment of one sorted scan; from-container, a packet's source program
 * and its local delivery draw on budgets of their own (source map, destination map),
 * and a pass is undone from a log of the CT slots it wrote.  An egress launch whose
 * passes find no fixed point, or that has no device memory for its saved state, runs
 * again in launches of as many packets as surely fit (one packet at the limit). */
int cv_ct_gc(cv_ctx *ctx, int h, uint32_t time, uint32_t *deleted);
/* Slot occupancy of a device CT map (diagnostics, no reference counterpart): out[0]
 * empty slots, out[1] tombstones (deleted entries not yet reclaimed by cv_ct_gc),
 * out[2] live entries. */
int cv_ct_slots(cv_ctx *ctx, int h, uint64_t out[3]);

/* ---- binding: programs -> maps ---- */
int cv_bind(cv_ctx *ctx, int role, int map_handle /* -1 unbinds */);
/* tail-call target cilium_policy[lxc_id] (maps.h:44-51): endpoint policy map and
 * CT_MAP4 (bpf_lxc.c:65-75).  Returns the endpoint index or -errno.  Its program
 * constants (LXC_IPV4, ...) and CT_MAP6 come from cv_endpoint_config. */
int cv_endpoint_add(cv_ctx *ctx, uint16_t lxc_id, uint32_t seclabel, int policy_map, int ct4_map);
/* the endpoint program's lxc_config.h constants (pkg/endpoint/bpf.go:152-200) and
 * its CT_MAP6 (bpf_lxc.c:53-63); addresses in network order.  ipv4 == 0: the
 * endpoint has no IPv4 programs (no LXC_IPV4). */
typedef struct {
    uint32_t ipv4;            /* LXC_IPV4, raw network-order word */
    uint8_t  ipv6[16];        /* LXC_IP */
    uint8_t  mac[6];          /* LXC_MAC */
    uint8_t  node_mac[6];     /* NODE_MAC */
    int      ct6_map;         /* ipv6_ct_tuple -> ct_entry map, or -1 */
} cv_endpoint_cfg;
int cv_endpoint_config(cv_ctx *ctx, int ep, const cv_endpoint_cfg *cfg);

/* node_config.h constants (raw network-order words; pkg/node/node_address.go) */
typedef struct {
    uint32_t ipv4_cluster_mask;   /* IPV4_CLUSTER_MASK  */
    uint32_t ipv4_cluster_range;  /* IPV4_CLUSTER_RANGE */
    uint32_t ipv4_loopback;       /* IPV4_LOOPBACK      */
    uint8_t  router_ip6[16];      /* ROUTER_IP          */
    uint8_t  host_mac[6];         /* HOST_IFINDEX_MAC   */
    uint8_t  net_mac[6];          /* CILIUM_NET_MAC: bpf_netdev's rewrite_dmac_to_host (FROM_HOST) */
} cv_node_cfg;
int cv_node_config(cv_ctx *ctx, const cv_node_cfg *cfg);

/* Make every pending map write visible to the next batch.  Every batch call does this
 * itself first (RCU-like visibility at batch granularity): the
 * agent's writes since the last batch are applied to the host images of the device
 * tables and the changed words published in the stream of the batch about to run
 * (batches already submitted see the old tables, later ones the new) -- ipcache v4
 * and v6 prefixes and policy entries without waiting for the device.  A write the
 * incremental path cannot apply (other maps, endpoint changes, /0, a table past 80 %
 * load) rebuilds the table after the submitted batches finish.  A context's batches
 * are ordered across streams on the device (no host wait).  -EPROTO (here and from
 * every later call): a conntrack stage of an earlier batch read a group-list word past
 * its launch (a corrupt list; the word is skipped, never dereferenced) -- the device
 * state is suspect, close the context. */
int cv_sync(cv_ctx *ctx);
/* publications of incremental writes so far, and rebuilds (boundaries that waited) */
int cv_publish_stats(cv_ctx *ctx, uint64_t *publications, uint64_t *rebuilds);

/* ---- batches ---- */
typedef struct {
    const uint8_t  *frames;   /* n records of `stride` bytes: the first bytes of each frame */
    uint32_t        stride;   /* 64 (IPv4) or 128 (IPv6) */
    const uint32_t *len;      /* skb->len / data_end - data per packet */
    const uint32_t *mark;     /* skb->mark per packet, or NULL (0) */
    uint32_t        n;
} cv_batch;

typedef struct {              /* any pointer may be NULL */
    uint8_t  *xdp;            /* XDP_DROP / XDP_PASS */
    int32_t  *ret;            /* tc result: DROP_* (<0), TC_ACT_OK, TC_ACT_REDIRECT, proxy port */
    uint32_t *identity;       /* resolved source security identity */
    uint8_t  *ct;             /* CT_NEW..CT_RELATED, or CV_CT_NONE */
    uint16_t *proxy;          /* proxy port (network order) of an L7 redirect, else 0 */
    uint8_t  *nl;             /* map lookups the path performed (algorithmic-bytes accounting) */
    uint8_t  *nu;             /* map entry writes the path performed */
    int32_t  *reason;         /* DROP_* code behind a TC_ACT_SHOT (the cilium_metrics reason), else 0 */
    uint8_t  *frames_out;     /* optional (cv_netdev_ingress, cv_lxc_egress): n records of the batch's
                                 stride: the frame after the datapath's rewrites (lb4_xlate, rev-NAT,
                                 ipv4_l3 TTL/MACs, with the kernel's checksum updates) for a
                                 forwarded IPv4 packet, else the input record */
} cv_out;

/* config 1: bpf_xdp.c xdp_start over the batch */
int cv_xdp_prefilter(cv_ctx *ctx, const cv_batch *b, cv_out *o, void *stream);
/* config 2: ingress verdict of a NEW flow at endpoint `ep` (identity resolution of
 * bpf_netdev.c:357-398 + policy_can_access_ingress, policy.h:139-163) */
int cv_policy_ingress(cv_ctx *ctx, int ep, const cv_batch *b, cv_out *o, void *stream);
/* config 3: [xdp_start ->] from_netdev -> handle_ipv4 -> endpoint ipv4_policy with
 * conntrack, in packet order semantics; `now` = bpf_ktime_get_sec() of the batch */
int cv_netdev_ingress(cv_ctx *ctx, const cv_batch *b, uint32_t now, int with_prefilter,
                      cv_out *o, void *stream);

/* config 5: from-container (bpf_lxc.c:672-716 handle_ingress -> tail_handle_ipv4/6)
 * of each packet's source endpoint: handle_ipv4_from_lxc / ipv6_l3_from_lxc with
 * lb4/lb6 service lookup and lb{4,6}_local, egress conntrack and policy, and local
 * delivery into the destination endpoint's policy program; direct routing.
 * src_ep[i] = endpoint index (cv_endpoint_add order) of packet i, or NULL: all from
 * ep0.  flow_hash[i] = the packet's get_hash_recalc() (the LB slave choice; the
 * kernel's is keyed by a boot-random secret, so it is an input).  `identity` out =
 * the destination identity (dstID), `ct` = the egress CT result.  IPv6 needs
 * records of >= 128 bytes.  Device pointers. */
int cv_lxc_egress(cv_ctx *ctx, const cv_batch *b, const uint16_t *src_ep, uint32_t ep0,
                  const uint32_t *flow_hash, uint32_t now, cv_out *o, void *stream);

/* Config 5 as ONE node across GPUs with endpoint-owned conntrack (per-endpoint CT maps,
 * bpf_lxc.c:53-75 CT_MAP4 / CT_MAP6 per program): a packet's source program
 * runs on its source endpoint's GPU and its local delivery -- the destination's
 * ipv4_policy / ipv6_policy on the destination's map -- on the destination's GPU.
 * cv_lxc_egress_split = cv_lxc_egress without running local deliveries: such a packet
 * ends with ret CV_E_DEFER and its 64-byte delivery record in deliver[i] (n x 64 B,
 * 16-B aligned device buffer; byte 24 (IPv4) / 48 (IPv6) holds the destination endpoint
 * index as a u16), identity / ct as for cv_lxc_egress.
 * cv_lxc_deliver runs the destination programs of n such records (all IPv4, or all IPv6
 * with v6 = 1) in record order per (destination map, address pair): ret, reason, proxy,
 * nl, nu are the packet's final outputs, identity / ct the source program's.  Next to
 * a map's max_entries both calls are admitted: creates succeed exactly as in packet
 * (record) order within the call.  The caller exchanges the records between GPUs (RCCL
 * all_to_all) and orders the calls so every map sees its operations in packet order
 * (cilium_amd/epnode.py orders them per (map, peer), exact while maps have room). */
#define CV_E_DEFER (-3)
int cv_lxc_egress_split(cv_ctx *ctx, const cv_batch *b, const uint16_t *src_ep, uint32_t ep0,
                        const uint32_t *flow_hash, uint32_t now, cv_out *o, uint8_t *deliver, void *stream);
int cv_lxc_deliver(cv_ctx *ctx, const uint8_t *records, uint32_t n, int v6, uint32_t now, cv_out *o,
                   void *stream);

/* ---- cilium_metrics (metrics.h:43-58): dense [256 reasons][4 dirs]{count, bytes} u64,
 * device resident.  Read sums it to host; the device pointer lets a caller reduce it
 * across GPUs (RCCL) without a copy; an external buffer may replace it. */
int cv_metrics_read(cv_ctx *ctx, uint64_t *out /* 2048 u64 */);
int cv_metrics_reset(cv_ctx *ctx);
uint64_t *cv_metrics_device_ptr(cv_ctx *ctx);
int cv_metrics_attach(cv_ctx *ctx, uint64_t *device_buf /* 2048 u64, or NULL = own */);

/* ---- drop notifications: send_drop_notify / __send_drop_notify (bpf/lib/drop.h:40-108)
 * A drop on the conntrack paths (cv_netdev_ingress, cv_lxc_egress) appends one record:
 * the 32-byte struct drop_notify the reference emits on cilium_events, followed by the
 * packet's index in the batch (the perf sample's payload is the first len_cap bytes of
 * that packet, which the caller holds).  `hash` is the batch's flow_hash where the
 * entry point takes one (the skb hash, get_hash_recalc), else 0.  Records are appended
 * in no particular order; *count counts every drop, also those past `capacity` (lost
 * samples, as with a full perf ring).  The caller zeroes *count when it drains. */
typedef struct cv_drop_notify {
    uint8_t  type;        /* CILIUM_NOTIFY_DROP = 1 */
    uint8_t  subtype;     /* -DROP_* */
    uint16_t source;      /* EVENT_SOURCE: LXC_ID of the endpoint program, 0 for bpf_netdev */
    uint32_t hash;
    uint32_t len_orig, len_cap;   /* skb->len, min(TRACE_PAYLOAD_LEN = 128, len) */
    uint32_t src_label, dst_label;   /* 16-bit fields of cb[1] = src << 16 | dst */
    uint32_t dst_id, ifindex;
    uint32_t packet;      /* index in the batch */
    uint32_t reserved;
} cv_drop_notify;
/* device buffers; records NULL detaches (drops are then only counted in cilium_metrics) */
int cv_notify_attach(cv_ctx *ctx, cv_drop_notify *records, uint32_t capacity, uint32_t *count);

/* ---- trace notifications: send_trace_notify (bpf/lib/trace.h:96-150, TRACE_NOTIFY on)
 * Every forwarding step of the conntrack paths appends one record: TRACE_FROM_STACK /
 * FROM_HOST / FROM_PROXY at from_netdev (bpf_netdev.c:478-492; ifindex = the
 * `ingress_ifindex` given here), TRACE_FROM_LXC at from-container (bpf_lxc.c:681),
 * TRACE_TO_LXC / TO_PROXY in ipv{4,6}_policy (:828-841, 956-971), TO_HOST / TO_STACK /
 * TO_PROXY at the from-container exits (:243-354, 542-645).  `aggregation` is
 * MONITOR_AGGREGATION (pkg/option/monitor.go: 0 none, 1 lowest, 2 low, 3 medium): >= 1
 * hides the FROM_* points, >= 3 keeps only steps whose conntrack lookup asked for a
 * report (ct_update_timeout's CT_REPORT_INTERVAL / new-flags logic, conntrack.h:103-161).
 * Same ring semantics as cv_notify_attach. */
typedef struct cv_trace_notify {
    uint8_t  type;        /* CILIUM_NOTIFY_TRACE = 4 */
    uint8_t  subtype;     /* TRACE_TO_LXC = 0 ... TRACE_FROM_OVERLAY = 9 */
    uint16_t source;      /* EVENT_SOURCE: LXC_ID of the endpoint program, 0 for bpf_netdev */
    uint32_t hash;
    uint32_t len_orig, len_cap;
    uint32_t src_label, dst_label;
    uint16_t dst_id;
    uint8_t  reason;      /* TRACE_REASON_* = the CT result (CT_NEW = 0 ... CT_RELATED = 3) */
    uint8_t  pad;
    uint32_t ifindex;
    uint32_t packet;      /* index in the batch */
    uint32_t reserved;
} cv_trace_notify;
int cv_trace_attach(cv_ctx *ctx, cv_trace_notify *records, uint32_t capacity, uint32_t *count,
                    uint32_t aggregation, uint32_t ingress_ifindex);

#ifdef __cplusplus
}
#endif
#endif
