/*
 * cilium_agent.h — host-side agent logic of the verdict path, over the C-ABI of
 * cilium_hip.h.
 *
 * The reference's agent (Go, pkg/) keeps two pieces of state machinery directly in
 * front of the maps this engine holds:
 *
 *  (1) the XDP prefilter's CIDR sets, with revisions and all-or-nothing batch
 *      updates (pkg/policy/prefilter.go:57-298 over pkg/maps/cidrmap/cidrmap.go);
 *  (2) an endpoint's policy map kept equal to its desired state, with the realized
 *      state tracked per key (Endpoint.syncPolicyMap, pkg/endpoint/endpoint.go:
 *      2515-2604, over pkg/maps/policymap/policymap.go:146-240).
 *
 * No Go toolchain exists in this image, so both are restated here in C++ (the
 * reference's host code is compiled code) and call the engine only through its
 * C-ABI map functions, as the Go code calls bpf(2) through pkg/bpf.  The maps they
 * write are the ones the datapath reads; writes reach the device at the next batch
 * boundary (cv_sync).  Errors are negative errnos plus, where the reference returns
 * a formatted error, its message in the caller's buffer.
 */
#ifndef CILIUM_AGENT_H
#define CILIUM_AGENT_H

#include <stdint.h>

#include "cilium_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- (1) prefilter (pkg/policy/prefilter.go) ---- */
typedef struct cv_prefilter cv_prefilter;

/* a net.IPNet: family 4 or 6, prefix length, address bytes in network order (v4:
 * addr[0..3]); the address is used as given, like cidrmap.cidrKeyInit (callers pass
 * the network address, as net.ParseCIDR returns it) */
typedef struct {
    uint8_t family;
    uint8_t prefixlen;
    uint8_t pad[2];
    uint8_t addr[16];
} cv_cidr;

/* the preFilterMapType order of prefilter.go:30-39 */
#define CV_PF_V4_DYN 0
#define CV_PF_V4_FIX 1
#define CV_PF_V6_DYN 2
#define CV_PF_V6_FIX 3

/* preFilterConfig bits */
#define CV_PF_DYN4 1
#define CV_PF_FIX4 2
#define CV_PF_DYN6 4
#define CV_PF_FIX6 8
#define CV_PF_DEFAULT (CV_PF_FIX4 | CV_PF_FIX6)   /* NewPreFilter (prefilter.go:281-298) */

/* NewPreFilter + init/initOneMap (prefilter.go:205-255, 281-298): revision 1; creates
 * the CIDR maps of the enabled config in ctx with cidrmap.OpenMapElems' shapes
 * (LPM_TRIE {u32 prefixlen, addr} -> u8 for the dyn maps, up to 64k; HASH for the fix
 * maps, up to 20M; BPF_F_NO_PREALLOC) and binds the ones the XDP program compiled
 * from WriteConfig reads to CV_ROLE_CIDR{4,6}_{FIX,DYN}.  The v6 fix map follows the
 * fix4 flag, as initOneMap does (prefilter.go:237). */
int  cv_prefilter_new(cv_ctx *ctx, uint32_t config, cv_prefilter **out);
void cv_prefilter_free(cv_prefilter *pf);
/* Insert / Delete (prefilter.go:125-203): a batch of CIDRs for `revision` (0 = any),
 * all or nothing (the applied part is undone on a failure), revision + 1 on success.
 * -ESTALE: revision mismatch; -EINVAL: no map enabled for a CIDR; -ENOENT (Delete):
 * a CIDR not in its map (checked before any change); else the failing map
 * operation's errno.  err (may be NULL) receives the reference's message. */
int cv_prefilter_insert(cv_prefilter *pf, int64_t revision, const cv_cidr *cidrs, uint32_t n,
                        char *err, uint32_t errlen);
int cv_prefilter_delete(cv_prefilter *pf, int64_t revision, const cv_cidr *cidrs, uint32_t n,
                        char *err, uint32_t errlen);
/* Dump (prefilter.go:91-106): the CIDRs of every map in map order, each map walked by
 * GetNextKey from the zero key (cidrmap.CIDRDump), and the current revision.  Returns
 * the number of CIDRs (up to cap written) or -errno. */
int cv_prefilter_dump(cv_prefilter *pf, cv_cidr *out, uint32_t cap, int64_t *revision);
/* WriteConfig (prefilter.go:65-89): the node-config #defines, NUL-terminated; returns
 * the length needed (excluding the NUL). */
int cv_prefilter_write_config(cv_prefilter *pf, char *buf, uint32_t len);
/* the map handle of CV_PF_*, or -1 when that map is not enabled */
int cv_prefilter_map(cv_prefilter *pf, int which);

/* ---- (2) policy map sync (pkg/endpoint/endpoint.go:2515-2604) ---- */
typedef struct cv_policy_sync cv_policy_sync;

/* policymap.PolicyKey in HOST byte order (PolicyMapState keys) */
typedef struct {
    uint32_t identity;
    uint16_t dport;
    uint8_t nexthdr;
    uint8_t direction;     /* 0 ingress, 1 egress */
} cv_policy_key;

int  cv_policy_sync_new(cv_policy_sync **out);
void cv_policy_sync_free(cv_policy_sync *s);
/* replaces desiredMapState: n keys with their proxy ports (host order) */
int cv_policy_sync_set_desired(cv_policy_sync *s, const cv_policy_key *keys, const uint16_t *proxy_ports,
                               uint32_t n);
/* syncPolicyMap: dumps policy map h (policymap.DumpToSlice: a GetNextKey walk from
 * the zero key, a lookup per key), deletes every key not desired (and from the
 * realized state), then writes every desired key whose realized entry is missing or
 * different (AllowKey: BPF_ANY, dport and proxy port to network order, counters 0)
 * and records it as realized.  Failed operations are counted and skipped.  Returns
 * 0, -EIO when some operation failed, or the dump's errno. */
int cv_policy_sync_run(cv_policy_sync *s, cv_ctx *ctx, int h, uint32_t *deleted, uint32_t *added,
                       uint32_t *failed);
/* realizedMapState: up to cap keys and proxy ports; returns the number of keys */
int cv_policy_sync_realized(cv_policy_sync *s, cv_policy_key *keys, uint16_t *proxy_ports, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif
