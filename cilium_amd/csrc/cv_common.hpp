// cv_common.hpp — constants shared by the host store, the table compiler and the
// gfx950 kernels.  Codes are the reference's (bpf/lib/common.h, bpf/include/bpf/api.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CV_HD __host__ __device__ __forceinline__
// Device pointers that come out of memory (the tables of an endpoint, read from the
// endpoint array) have no address space the compiler can see, so their accesses
// become flat instructions (the address-space check, and a wait on both the vector
// and the LDS/scalar counters at every use).  G() states that a pointer is global.
#if defined(__HIP_DEVICE_COMPILE__)
#define CV_G __attribute__((address_space(1)))
#else
#define CV_G
#endif
template <class T>
__host__ __device__ __forceinline__ CV_G T *G(T *p) { return (CV_G T *)p; }

namespace cv {

// bpf/lib/common.h:237-269
enum : int32_t {
    DROP_INVALID_SMAC = -130, DROP_INVALID_DMAC = -131, DROP_INVALID_SIP = -132,
    DROP_POLICY = -133, DROP_INVALID = -134, DROP_CT_INVALID_HDR = -135,
    DROP_CT_UNKNOWN_PROTO = -137, DROP_UNKNOWN_L3 = -139, DROP_MISSED_TAIL_CALL = -140,
    DROP_WRITE_ERROR = -141, DROP_UNKNOWN_L4 = -142, DROP_CSUM_L3 = -153, DROP_CSUM_L4 = -154,
    DROP_CT_CREATE_FAILED = -155,
    DROP_INVALID_EXTHDR = -156, DROP_FRAG_NOSUPPORT = -157, DROP_NO_SERVICE = -158,
};
// E_TRUNC: a byte the path reads lies beyond the record (the caller must hand over
// more of the frame); E_PUNT: the packet left the path through a tail call into a
// responder program (ARP, ICMPv6 NS / echo-to-router / hop limit); E_FAULT: the
// -EFAULT of a failed skb_load_bytes(), which the reference treats as a drop code.
enum : int32_t { TC_ACT_OK = 0, TC_ACT_SHOT = 2, TC_ACT_REDIRECT = 7, E_TRUNC = -1, E_PUNT = -2, E_DEFER = -3,
                 E_FAULT = -14 };
enum : uint8_t { XDP_DROP = 1, XDP_PASS = 2 };
enum : uint8_t { CT_NEW = 0, CT_ESTABLISHED = 1, CT_REPLY = 2, CT_RELATED = 3, CT_NONE = 0xff };
enum : int { CT_EGRESS = 0, CT_INGRESS = 1, CT_SERVICE = 2 };

// bpf/node_config.h
constexpr uint32_t HOST_ID = 1, WORLD_ID = 2, CLUSTER_ID = 3, HEALTH_ID = 4, HOST_IFINDEX = 1;

// datapath option bits (include/cilium_hip.h CV_F_*)
constexpr uint32_t F_FROM_HOST = 0x1, F_HAVE_L4_POLICY = 0x2, F_DROP_ALL = 0x4, F_CT_ACCOUNTING = 0x8,
                   F_POLICY_INGRESS = 0x10, F_POLICY_EGRESS = 0x20;
// test hook (CV_COARSE_GROUPS, cv_ctx.cpp params): the netdev front keeps 8 bits of every
// group key, so groups of different address pairs and CT maps merge into long runs (a
// coarser grouping is equally exact: DESIGN.md §4)
constexpr uint32_t F_TEST_COARSE_GROUPS = 0x80000000u;
// CV_F_ACCT_SPLIT (include/cilium_hip.h): nl / nu count conntrack lookups and writes
// ACCT_CT_UNIT each (cv_dev.hpp), for the HBM-resident split of the algorithmic bytes
constexpr uint32_t F_ACCT_SPLIT = 0x40;

// conntrack.h:31-66
constexpr uint32_t CT_LIFETIME_TCP = 21600, CT_LIFETIME_NONTCP = 60, CT_SYN_TIMEOUT = 60,
                   CT_CLOSE_TIMEOUT = 10, CT_REPORT_INTERVAL = 5;
constexpr uint8_t TUPLE_F_OUT = 0, TUPLE_F_IN = 1, TUPLE_F_RELATED = 2, TUPLE_F_SERVICE = 4;
// ct_entry u16 bitfield at offset 36 (common.h:386-391)
constexpr uint16_t CTB_RX_CLOSING = 0x1, CTB_TX_CLOSING = 0x2, CTB_NAT46 = 0x4, CTB_LB_LOOPBACK = 0x8,
                   CTB_SEEN_NON_SYN = 0x10;
constexpr uint8_t TCPF_FIN = 0x01, TCPF_SYN = 0x02, TCPF_RST = 0x04;

// metrics (common.h:195-206, 271-278): dense [256][4]{count, bytes}
constexpr int METRICS_WORDS = 256 * 4 * 2;
constexpr uint8_t METRIC_INGRESS = 1, METRIC_EGRESS = 2;

CV_HD uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
CV_HD uint16_t bswap16(uint16_t x) { return __builtin_bswap16(x); }

// 64-bit finalizer (splitmix64) over key words
CV_HD uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

template <int KW>
CV_HD uint64_t hash_words(const uint32_t *k, uint64_t seed)
{
    uint64_t h = seed;
#pragma unroll
    for (int i = 0; i < KW; i += 2) {
        uint64_t w = k[i] | (i + 1 < KW ? (uint64_t)k[i + 1] << 32 : 0);
        h = mix64(h ^ w) + 0x9E3779B97F4A7C15ULL;
    }
    return mix64(h);
}

}  // namespace cv
