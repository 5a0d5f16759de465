/*
 * ref_probe.c — links the reference's own pure helpers and struct definitions
 * (compiled from /root/reference/bpf where they lie; nothing is copied) so the
 * oracle's restatements can be checked against them.  TEST INFRASTRUCTURE.
 * Only pure code is used: no BPF helper is called.
 */
#include <stddef.h>
#include <stdint.h>
#include "lib/utils.h"
#include "node_config.h"
#include "lib/common.h"
#include "lib/ipv6.h"
#include "lib/maps.h"
#include "lib/xdp.h"

uint32_t ref_get_prefix(int prefix) { return GET_PREFIX(prefix); }

void ref_ipv6_addr_clear_suffix(uint8_t addr[16], int prefix)
{
    union v6addr a;
    __builtin_memcpy(&a, addr, 16);
    ipv6_addr_clear_suffix(&a, prefix);
    __builtin_memcpy(addr, &a, 16);
}

/* name, sizeof, then offsets of interest; returned as a flat table */
#define L(s) sizeof(struct s)
long ref_layout(int i)
{
    static const long t[] = {
        L(lpm_v4_key), L(lpm_v6_key), L(lpm_val), L(endpoint_key), L(endpoint_info),
        L(ipcache_key), L(remote_endpoint_info), L(policy_key), L(policy_entry),
        L(metrics_key), L(metrics_value), L(ipv4_ct_tuple), L(ipv6_ct_tuple), L(ct_entry),
        L(lb4_key), L(lb4_service), L(lb6_key), L(lb6_service),
        offsetof(struct endpoint_key, family), offsetof(struct endpoint_info, lxc_id),
        offsetof(struct endpoint_info, flags), offsetof(struct ipcache_key, family),
        offsetof(struct ipcache_key, ip4), offsetof(struct policy_entry, packets),
        offsetof(struct ipv4_ct_tuple, dport), offsetof(struct ipv4_ct_tuple, nexthdr),
        offsetof(struct ct_entry, lifetime), offsetof(struct ct_entry, rev_nat_index),
        offsetof(struct ct_entry, slave), offsetof(struct ct_entry, tx_flags_seen),
        offsetof(struct ct_entry, rx_flags_seen), offsetof(struct ct_entry, src_sec_id),
        offsetof(struct ct_entry, last_tx_report), offsetof(struct ct_entry, last_rx_report),
        offsetof(struct ipv6_ct_tuple, dport), offsetof(struct ipv6_ct_tuple, nexthdr),
    };
    if (i < 0) return (long)(sizeof(t) / sizeof(t[0]));
    return t[i];
}

/* ct_entry bitfield positions inside the u16 at offset 36 */
int ref_ct_bit(int which)
{
    struct ct_entry e; __builtin_memset(&e, 0, sizeof(e));
    switch (which) {
    case 0: e.rx_closing = 1; break;
    case 1: e.tx_closing = 1; break;
    case 2: e.nat46 = 1; break;
    case 3: e.lb_loopback = 1; break;
    case 4: e.seen_non_syn = 1; break;
    }
    uint16_t v; __builtin_memcpy(&v, (char *)&e + 36, 2);
    return v;
}

/* policy_key egress bit position inside byte 7 */
int ref_policy_egress_byte(void)
{
    struct policy_key k; __builtin_memset(&k, 0, sizeof(k));
    k.egress = 1;
    return ((unsigned char *)&k)[7];
}
