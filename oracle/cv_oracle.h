/*
 * cv_oracle.h — CPU restatement of Cilium's L3/L4 verdict path (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for the MI355X verdict engine.  It is NOT product
 * code: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker.  The product library (cilium_amd/) never
 * links or calls anything under oracle/.
 *
 * Every function restates a function of the reference (Taeung/cilium v1.1.90,
 * /root/reference) and cites the file:line it follows.  Kernel map semantics
 * (HASH / LRU_HASH / LPM_TRIE from Linux kernel/bpf/{hashtab,lpm_trie}.c, a
 * third-party dependency absent from the reference) are restated from their
 * published behaviour and pinned against the container kernel's own maps
 * (oracle/kernel_golden.py -> tests/golden/).
 */
#ifndef CV_ORACLE_H
#define CV_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- BPF map types / flags (include/linux/bpf.h in the reference) ---- */
#define OR_MAP_HASH      1
#define OR_MAP_LRU_HASH  9
#define OR_MAP_LPM_TRIE 11
#define OR_BPF_ANY       0
#define OR_BPF_NOEXIST   1
#define OR_BPF_EXIST     2

/* ---- return codes (bpf/include/bpf/api.h:18-25, include/linux/bpf.h:623-628) */
#define OR_TC_ACT_OK        0
#define OR_TC_ACT_SHOT      2
#define OR_TC_ACT_REDIRECT  7
#define OR_XDP_DROP 1
#define OR_XDP_PASS 2

/* ---- datapath drop codes (bpf/lib/common.h:237-269) */
#define OR_DROP_INVALID_SMAC      -130
#define OR_DROP_INVALID_DMAC      -131
#define OR_DROP_INVALID_SIP       -132
#define OR_DROP_POLICY            -133
#define OR_DROP_INVALID           -134
#define OR_DROP_CT_INVALID_HDR    -135
#define OR_DROP_CT_UNKNOWN_PROTO  -137
#define OR_DROP_UNKNOWN_L3        -139
#define OR_DROP_MISSED_TAIL_CALL  -140
#define OR_DROP_UNKNOWN_L4        -142
#define OR_DROP_NO_LXC            -152
#define OR_DROP_CT_CREATE_FAILED  -155
#define OR_DROP_INVALID_EXTHDR    -156
#define OR_DROP_FRAG_NOSUPPORT    -157
#define OR_DROP_NO_SERVICE        -158
#define OR_DROP_CSUM_L3 (-153)
#define OR_DROP_CSUM_L4 (-154)
#define OR_DROP_WRITE_ERROR       -141
#define OR_DROP_PROXYMAP_CREATE_FAILED -159
/* oracle-only: a header byte the reference would read lies beyond the record */
#define OR_E_TRUNC                -1
/* oracle-only: the packet left this path through a tail call into a responder
 * program outside it (ARP / ICMPv6 NS / echo-to-router / hop-limit-exceeded) */
#define OR_E_PUNT                 -2
/* oracle-internal, never an output: a load_byte() (BPF_LD_ABS) past the packet ended
 * the program, which then returns 0 (TC_ACT_OK) with no notification */
#define OR_E_LDABS                -3
/* skb_load_bytes() failure as the BPF helper reports it (-EFAULT) */
#define OR_E_FAULT                -14

/* CT results (bpf/lib/common.h:331-336) */
#define OR_CT_NEW 0
#define OR_CT_ESTABLISHED 1
#define OR_CT_REPLY 2
#define OR_CT_RELATED 3
#define OR_CT_NONE 0xff

/* CT directions (bpf/lib/common.h:327-329) */
#define OR_CT_EGRESS  0
#define OR_CT_INGRESS 1
#define OR_CT_SERVICE 2

/* ---- key/value layouts (bpf/lib/common.h, bpf/lib/maps.h, bpf/lib/xdp.h) */
#pragma pack(push, 1)
typedef struct { uint32_t prefixlen; uint8_t addr[4]; } or_lpm_v4_key;    /* xdp.h:23-26 */
typedef struct { uint32_t prefixlen; uint8_t addr[16]; } or_lpm_v6_key;   /* xdp.h:28-31 */
typedef struct { uint8_t ip[16]; uint8_t family; uint8_t pad4; uint16_t pad5; } or_endpoint_key; /* common.h:147-160 */
typedef struct { uint32_t prefixlen; uint8_t pad[3]; uint8_t family; uint8_t ip[16]; } or_ipcache_key; /* maps.h:135-148 */
typedef struct { uint32_t daddr, saddr; uint16_t dport, sport; uint8_t nexthdr, flags; } or_ipv4_ct_tuple; /* common.h:359-367 */
typedef struct { uint32_t address; uint16_t dport; uint16_t slave; } or_lb4_key;                /* common.h:427-431 */
typedef struct { uint32_t target; uint16_t port; uint16_t count; uint16_t rev_nat_index; uint16_t weight; } or_lb4_service; /* common.h:433-439 */
typedef struct { uint8_t address[16]; uint16_t dport; uint16_t slave; } or_lb6_key;             /* common.h:408-412 */
typedef struct { uint8_t target[16]; uint16_t port; uint16_t count; uint16_t rev_nat_index; uint16_t weight; } or_lb6_service; /* common.h:414-420 */
#pragma pack(pop)

typedef struct {             /* common.h:165-173, 48 bytes: mac_t is 8-byte aligned (mac @16) */
    uint32_t ifindex; uint16_t unused; uint16_t lxc_id; uint32_t flags; uint32_t pad0;
    uint8_t mac[8], node_mac[8]; uint32_t pad[4];
} or_endpoint_info;
typedef struct { uint32_t sec_label; uint32_t tunnel_endpoint; } or_remote_endpoint_info; /* common.h:175-178 */
typedef struct { uint32_t sec_label; uint16_t dport; uint8_t protocol; uint8_t egress_pad; } or_policy_key; /* common.h:180-186 */
typedef struct { uint16_t proxy_port; uint16_t pad[3]; uint64_t packets; uint64_t bytes; } or_policy_entry;  /* common.h:188-193 */
typedef struct {             /* common.h:380-406, 56 bytes; bits@36: rx_closing b0, tx_closing b1, nat46 b2, lb_loopback b3, seen_non_syn b4 */
    uint64_t rx_packets, rx_bytes, tx_packets, tx_bytes;
    uint32_t lifetime; uint16_t bits; uint16_t rev_nat_index; uint16_t slave;
    uint8_t tx_flags_seen, rx_flags_seen; uint32_t src_sec_id; uint32_t last_tx_report, last_rx_report;
} or_ct_entry;
typedef struct {             /* common.h:452-461 (internal) */
    uint16_t rev_nat_index; uint16_t loopback; uint16_t orig_dport; uint32_t addr, svc_addr, src_sec_id; uint16_t slave;
} or_ct_state;
typedef struct {             /* common.h:338-346, 40 bytes, unpacked: 2 zero pad bytes */
    uint8_t daddr[16], saddr[16]; uint16_t dport, sport; uint8_t nexthdr, flags; uint16_t pad;
} or_ipv6_ct_tuple;
#pragma pack(push, 1)
typedef struct { uint32_t address; uint16_t port; } or_lb4_reverse_nat;       /* common.h:441-444 */
typedef struct { uint8_t address[16]; uint16_t port; } or_lb6_reverse_nat;    /* common.h:422-425 */
#pragma pack(pop)

/* ---- generic kernel-semantics map ---- */
typedef struct or_map or_map;
or_map  *or_map_create(int type, uint32_t key_size, uint32_t val_size, uint32_t max_entries);
void     or_map_free(or_map *m);
int      or_map_update(or_map *m, const void *key, const void *val, uint64_t flags);
int      or_map_update_batch(or_map *m, const void *keys, const void *vals, uint32_t n, uint64_t flags);
int      or_map_lookup(or_map *m, const void *key, void *val_out);
int      or_map_delete(or_map *m, const void *key);
uint32_t or_map_count(const or_map *m);
/* all entries, sorted by key bytes; returns the count written (<= max) */
uint32_t or_map_dump(const or_map *m, void *keys, void *vals, uint32_t max);
void or_map_digest(const or_map *m, uint64_t out[3]);   /* test infrastructure */
/* nl / nu: conntrack lookups and writes count 32 (CV_F_ACCT_SPLIT's split), or 1 */
void or_set_acct_split(int on);
/* the kernel checksum helper restatement (known-answer tests) */
int or_csum_apply(uint8_t *frame, uint32_t len, uint32_t op, uint32_t off, uint32_t from, uint32_t to,
                  uint32_t flags, uint64_t *diff);
/* ctmap.GC(GCFilterByTime) on a CT map: delete entries with lifetime < time */
uint32_t or_ct_gc(or_map *m, uint32_t time);
void    *or_map_lookup_ptr(or_map *m, const void *key);

/* ---- restated helpers pinned by test/bpf/unit-test.c ---- */
uint32_t or_get_prefix(int prefix);                               /* ipv6.h:136-138 (GET_PREFIX) */
void     or_ipv6_addr_clear_suffix(uint8_t addr[16], int prefix); /* ipv6.h:140-150 */

/* ---- datapath configuration ---- */
#define OR_F_FROM_HOST      0x1   /* bpf_netdev.c built with netdev_config.h FROM_HOST */
#define OR_F_HAVE_L4_POLICY 0x2   /* lxc_config.h HAVE_L4_POLICY */
#define OR_F_DROP_ALL       0x4   /* pkg/endpoint/bpf.go DROP_ALL */
#define OR_F_CT_ACCOUNTING  0x8   /* CONNTRACK_ACCOUNTING (daemon/main.go:676 default on) */
#define OR_F_POLICY_INGRESS 0x10  /* POLICY_INGRESS */
#define OR_F_POLICY_EGRESS  0x20  /* POLICY_EGRESS */
#define OR_F_DEFAULT (OR_F_FROM_HOST | OR_F_HAVE_L4_POLICY | OR_F_CT_ACCOUNTING | OR_F_POLICY_INGRESS | OR_F_POLICY_EGRESS)

#define OR_MAX_EP 8192
typedef struct {
    uint16_t lxc_id; uint32_t seclabel;
    or_map *policy;          /* cilium_policy_<id> */
    or_map *ct4;             /* CT_MAP4 of this endpoint (may be a shared global map) */
    or_map *ct6;             /* CT_MAP6 (bpf_lxc.c:53-63) */
    /* lxc_config.h constants of the endpoint's program (pkg/endpoint/bpf.go:152-200) */
    uint32_t ipv4;           /* LXC_IPV4 (raw, network order); 0 = no IPv4 program */
    uint8_t  ipv6[16];       /* LXC_IP */
    uint8_t  mac[6];         /* LXC_MAC */
    uint8_t  node_mac[6];    /* NODE_MAC */
} or_endpoint_prog;

/* struct drop_notify (bpf/lib/drop.h:40-48) + the packet's batch index */
typedef struct {
    uint8_t  type, subtype;
    uint16_t source;
    uint32_t hash, len_orig, len_cap, src_label, dst_label, dst_id, ifindex, packet, reserved;
} or_drop_notify;

/* struct trace_notify (bpf/lib/trace.h:72-82) + the packet's batch index */
typedef struct {
    uint8_t  type, subtype;
    uint16_t source;
    uint32_t hash, len_orig, len_cap, src_label, dst_label;
    uint16_t dst_id;
    uint8_t  reason, pad;
    uint32_t ifindex, packet, reserved;
} or_trace_notify;

typedef struct or_dp {
    /* prefilter (bpf_xdp.c); NULL disables the map (filter_config.h) */
    or_map *v4_fix, *v4_dyn, *v6_fix, *v6_dyn;
    or_map *lxc;             /* cilium_lxc  (maps.h:27-33) */
    or_map *ipcache;         /* cilium_ipcache (maps.h:151-158) */
    or_map *lb4_services, *lb6_services;
    or_map *lb4_revnat, *lb6_revnat;   /* cilium_lb{4,6}_reverse_nat (lb.h:37-68) */
    uint32_t flags;
    /* node_config.h constants (raw network-order words) */
    uint32_t v4_cluster_mask, v4_cluster_range, v4_loopback;
    uint8_t  router_ip6[16];
    uint8_t  host_mac[6];             /* HOST_IFINDEX_MAC */
    uint8_t  net_mac[6];              /* CILIUM_NET_MAC (node_config.h:57): rewrite_dmac_to_host */
    uint32_t n_ep;
    or_endpoint_prog ep[OR_MAX_EP];   /* tail-call targets of cilium_policy (maps.h:44-51) */
    uint16_t ep_of_lxc[65536];        /* lxc_id -> index + 1 */
    uint64_t metrics[256][4][2];      /* Σ over CPUs of cilium_metrics (metrics.h:43-58): [reason][dir]{count,bytes} */
    /* cilium_events drop notifications (DROP_NOTIFY), when attached */
    or_drop_notify *notify;
    uint32_t notify_cap, notify_n;
    or_trace_notify *trace;           /* send_trace_notify records (NULL: metrics only) */
    uint32_t trace_cap, trace_n;
    uint32_t trace_agg;               /* MONITOR_AGGREGATION (pkg/option/monitor.go levels 0-3) */
    uint32_t ingress_ifindex;         /* skb->ingress_ifindex of from_netdev */
    uint32_t cur_pkt, cur_hash;       /* the packet being processed and its skb hash */
    /* or_lxc_egress_split: stop a packet at its local delivery, recording where it goes */
    int32_t  split;
    int32_t  pend_ep;                 /* the destination endpoint's index (-1: none) */
    uint32_t pend_ifindex, pend_label;
} or_dp;

or_dp *or_dp_create(uint32_t flags);
void   or_dp_free(or_dp *dp);          /* does not free maps */
int    or_dp_add_endpoint(or_dp *dp, uint16_t lxc_id, uint32_t seclabel, or_map *policy, or_map *ct4);
/* the endpoint program's lxc_config.h constants and its CT_MAP6 */
int    or_dp_endpoint_config(or_dp *dp, uint32_t ep, uint32_t ipv4, const uint8_t *ipv6, const uint8_t *mac,
                             const uint8_t *node_mac, or_map *ct6);
/* node_config.h: IPV4_CLUSTER_MASK / IPV4_CLUSTER_RANGE / IPV4_LOOPBACK / ROUTER_IP /
 * HOST_IFINDEX_MAC / CILIUM_NET_MAC (NULL macs leave them zero) */
void   or_dp_node_config(or_dp *dp, uint32_t v4_cluster_mask, uint32_t v4_cluster_range, uint32_t v4_loopback,
                         const uint8_t *router_ip6, const uint8_t *host_mac, const uint8_t *net_mac);
void   or_dp_metrics(const or_dp *dp, uint64_t *out /* [256][4][2] */);
/* attach a record buffer (NULL detaches); returns and resets nothing: see or_dp_notify_count */
void   or_dp_notify_attach(or_dp *dp, or_drop_notify *buf, uint32_t cap);
uint32_t or_dp_notify_count(const or_dp *dp);
/* attach a trace record buffer (NULL detaches) with the aggregation level and the
 * netdev's ingress ifindex */
void   or_dp_trace_attach(or_dp *dp, or_trace_notify *buf, uint32_t cap, uint32_t aggregation,
                          uint32_t ingress_ifindex);
uint32_t or_dp_trace_count(const or_dp *dp);

/* per-packet outputs (SoA; any pointer may be NULL) */
typedef struct {
    uint8_t  *xdp;        /* XDP verdict (1 drop / 2 pass) */
    int32_t  *ret;        /* tc verdict: negative DROP_*, TC_ACT_OK, TC_ACT_REDIRECT */
    uint32_t *identity;   /* resolved source identity */
    uint8_t  *ct;         /* CT result or OR_CT_NONE */
    uint16_t *proxy;      /* proxy port (raw be16) when redirected to proxy */
    uint8_t  *nl;         /* map lookups performed (algorithmic bytes) */
    uint8_t  *nu;         /* map entry writes performed */
    int32_t  *reason;     /* DROP_* behind a TC_ACT_SHOT, else 0 */
    uint8_t  *frames_out; /* the frame after the datapath's rewrites (stride bytes per packet;
                             forwarded IPv4 packets; others: the input frame) */
} or_out;

/* Config 1: bpf_xdp.c xdp_start over a batch of frames (records of `stride` bytes). */
void or_xdp_prefilter(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                      uint32_t n, or_out *out);

/* Config 2: ingress verdict of a NEW flow for one endpoint: netdev identity resolution
 * (bpf_netdev.c:357-398) + policy_can_access_ingress (policy.h:139-163) with the L4
 * key as ct_lookup4 leaves it (conntrack.h:442-562) on a CT miss.  Parallel (OpenMP)
 * with atomic policy counters. */
void or_policy_ingress(or_dp *dp, uint32_t ep_index, const uint8_t *frames, uint32_t stride,
                       const uint32_t *len, const uint32_t *mark, uint32_t n, or_out *out);

/* Config 3: full ingress path: [XDP prefilter] -> from_netdev -> handle_ipv4 (tail call)
 * or handle_ipv6 -> tail call into the endpoint's ipv{4,6}_policy (CT lookup/create,
 * policy).  Sequential, as one CPU. */
void or_netdev_ingress(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                       const uint32_t *mark, uint32_t n, uint32_t now, int with_prefilter, or_out *out);

/* Config 5: from-container (bpf_lxc.c:672-716 handle_ingress) of the packets' source
 * endpoints: handle_ipv4_from_lxc / ipv6_l3_from_lxc with lb4/lb6 service lookup,
 * lb{4,6}_local, egress conntrack and policy, and local delivery into the destination
 * endpoint's ipv{4,6}_policy.  Sequential, as one CPU.  src_ep[i] = endpoint index
 * of packet i (NULL: all from ep0); flow_hash[i] = get_hash_recalc() of packet i. */
void or_lxc_egress(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                   const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash, uint32_t n,
                   uint32_t now, or_out *out);

/* Config 5 split at the local delivery, for the endpoint-owned CT prototype
 * (tests/ep_shard.py): as or_lxc_egress, but a packet whose program reaches a local
 * endpoint's policy program (ipv{4,6}_local_delivery -> tail call) stops there:
 * ret = OR_E_DEFER, dl_ep[i] = the destination endpoint's index (else -1), dl_ifindex /
 * dl_label = its ifindex and the source's seclabel, frames_out[i] the frame as the
 * source's program left it.  or_lxc_deliver then runs the destination programs of such
 * packets (pkt[j]: the batch index for notifications; nl / nu add to what out holds). */
#define OR_E_DEFER (-3)
void or_lxc_egress_split(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len,
                         const uint16_t *src_ep, uint32_t ep0, const uint32_t *flow_hash, uint32_t n,
                         uint32_t now, or_out *out, int32_t *dl_ep, uint32_t *dl_ifindex, uint32_t *dl_label);
void or_lxc_deliver(or_dp *dp, const uint8_t *frames, uint32_t stride, const uint32_t *len, const int32_t *dl_ep,
                    const uint32_t *dl_ifindex, const uint32_t *dl_label, const uint32_t *pkt, uint32_t n,
                    uint32_t now, or_out *out);

/* ct_create4 on a given tuple (conntrack.h:663-744), for building preloaded tables. */
int or_ct_create4(or_map *ct, or_ipv4_ct_tuple *tuple, uint32_t skb_len, int dir,
                  const or_ct_state *st, uint32_t now);
/* ct_lookup4 on a frame (conntrack.h:442-562); tuple in/out. */
int or_ct_lookup4(or_map *ct, or_ipv4_ct_tuple *tuple, const uint8_t *frame, uint32_t avail,
                  uint32_t len, int l4_off, int dir, or_ct_state *st, uint32_t now, uint32_t flags,
                  uint8_t *nl, uint8_t *nu);

/* lb4_lookup_service (lb.h:604-635) */
const or_lb4_service *or_lb4_lookup_service(or_map *svc_map, or_lb4_key *key, uint8_t *nl);

#ifdef __cplusplus
}
#endif
#endif
