/*
 * cilium_epnode.h — the round scheduler of config 5 as ONE node across GPUs with
 * endpoint-owned conntrack, over cv_lxc_egress_split / cv_lxc_deliver.
 *
 * The reference can give every endpoint its own CT maps: CT_MAP4 / CT_MAP6 are
 * per-program macros (bpf/bpf_lxc.c:52-75), per-endpoint maps when the endpoint's
 * conntrack is local (ConntrackLocal, pkg/endpoint/bpf.go:182-190; 64 000 entries,
 * pkg/maps/ctmap/ctmap.go:54).  Rank r owns the endpoints e with e % world == r and their
 * maps.  A packet's source program (handle_ipv4_from_lxc / ipv6_l3_from_lxc: the service
 * lookup and lb{4,6}_local, the egress conntrack and policy, bpf_lxc.c:402-649) runs on its
 * source's rank; its local delivery -- the destination's ipv4_policy / ipv6_policy on the
 * destination's map (bpf_lxc.c:721-1038) -- on the destination's rank, from the 64-B
 * record the source program hands over.
 *
 * The sequential answer is reproduced because every operation of a CT map keeps packet
 * order with the operations of that map it can interact with:
 *  - an entry of an endpoint's map is keyed by the endpoint's address and one peer, so
 *    operations sharing no peer touch disjoint entries; an operation waits for the
 *    earlier pending operations of its map that share a peer (the peers of a packet are
 *    supersets from its headers and the read-only service table);
 *  - next to max_entries the creates of DIFFERENT peers compete for the map's room
 *    (a create that finds the map full fails: DROP_CT_CREATE_FAILED,
 *    bpf/lib/conntrack.h:692-693), so a map that may fill -- live entries plus the creates
 *    its pending operations may still make (at most 7 per source program, 2 per delivery)
 *    exceed max_entries -- orders ALL its operations in packet order, across peers.
 * Within one launch the library keeps packet order per address pair and, next to a
 * limit, per map (admission), so a round launches every operation that no earlier
 * pending one blocks.
 *
 * Host-side scheduler (C++); the batches, records and outputs stay on the device.  A round:
 *   1. cv_epnode_sources      -> the source programs to launch (packet indices, ascending);
 *   2. (caller) cv_lxc_egress_split over them; the destination of each deferred packet;
 *   3. cv_epnode_sources_done -> the exchange rows: per launched packet and candidate
 *      destination, the record (or "not for you") for the destination's owner rank;
 *   4. (caller) the exchange (RCCL all_to_all of the rows and their 64-B records);
 *   5. cv_epnode_receive      -> per arriving row the delivery operation its record is for;
 *   6. cv_epnode_deliveries   -> the deliveries to launch (packet order); the caller runs
 *      cv_lxc_deliver over their records.
 * Errors are negative errnos; -EPROTO: a source program delivered outside the packet's
 * candidates, or a row names no delivery operation of this rank.
 */
#ifndef CILIUM_EPNODE_H
#define CILIUM_EPNODE_H

#include <stdint.h>

#include "cilium_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cv_epnode cv_epnode;

/* One batch of one rank.  frames: HOST copy of the n records (stride bytes each, IPv4
 * and IPv6 mixed: the ethertype decides); src_ep: the source endpoint of each packet
 * (cv_endpoint_add index).  The node's endpoints, their CT maps, the service table and
 * the loopback address come from ctx (every rank's ctx holds the same agent writes);
 * every endpoint's CT4 / CT6 map must be its own (-EINVAL otherwise). */
int  cv_epnode_open(cv_ctx *ctx, uint32_t rank, uint32_t world, const uint8_t *frames, uint32_t stride,
                    uint32_t n, const uint16_t *src_ep, cv_epnode **out);
void cv_epnode_close(cv_epnode *nd);

/* Where the scheduler reads the live entries and max_entries of CT maps (by handle) to
 * tell which maps may fill: by default the context's own maps (after the batches already
 * submitted); a caller holding the maps elsewhere supplies them.  Before the first round. */
typedef int (*cv_epnode_counts_fn)(void *arg, const int *handles, uint32_t n, uint64_t *live, uint64_t *max_entries);
int cv_epnode_set_counts(cv_epnode *nd, cv_epnode_counts_fn fn, void *arg);

/* operations of this rank not yet run or resolved */
uint64_t cv_epnode_pending(const cv_epnode *nd);

/* stats[0] rounds (calls of cv_epnode_sources), [1] source operations, [2] delivery
 * operations of this rank, [3] maps that were ordered whole (may fill) at open,
 * [4] those still so at the last round, [5] exchange rows sent to other ranks */
int cv_epnode_stats(const cv_epnode *nd, uint64_t stats[6]);

/* the round's source programs: packet indices, ascending (at most n); returns the count */
int cv_epnode_sources(cv_epnode *nd, uint32_t *pkts, uint32_t cap);

/* dst[j]: the destination endpoint of launched packet pkts[j] (its record at
 * deliver[j] of the split launch), or -1 when the source program ended it.  Writes the
 * exchange rows sorted by owner rank -- row_pkt, row_ep (the candidate), row_has (1: the
 * record is for row_ep), row_pos (j: where the record is), row_rank -- and per rank
 * the row count (rank_rows[world]); returns the number of rows (cap: at least
 * n x (candidates + 1) of the launched packets). */
int cv_epnode_sources_done(cv_epnode *nd, const uint32_t *pkts, const int32_t *dst, uint32_t n,
                           uint32_t *row_pkt, uint32_t *row_ep, uint8_t *row_has, uint32_t *row_pos,
                           uint32_t *rank_rows, uint32_t cap);

/* rows arriving at this rank (from every rank, itself included): op[j] = the delivery
 * operation whose record row j carries (the caller files the record under it), or -1
 * (the packet is not delivered here) */
int cv_epnode_receive(cv_epnode *nd, const uint32_t *row_pkt, const uint32_t *row_ep, const uint8_t *row_has,
                      uint32_t n, int32_t *op);

/* the round's deliveries: operation ids (as cv_epnode_receive named them) and their
 * packets, in packet order; returns the count */
int cv_epnode_deliveries(cv_epnode *nd, uint32_t *ops, uint32_t *pkts, uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif
