// cv_node.hpp — what the endpoint-owned node's scheduler (cv_epnode.cpp) reads from a
// context: the endpoints' addresses and CT maps, the service table's VIP -> backend
// pairs and the loopback address, as the agent wrote them (host images), and the live
// counts of conntrack maps (device-authoritative).  Internal to the library.
#pragma once
#include <stdint.h>

#include <vector>

struct cv_ctx;

namespace cv {

struct NodeEndpoint {
    uint32_t ipv4;             // LXC_IPV4, raw network-order word (0: none)
    uint8_t ipv6[16];          // LXC_IP (all zero: none)
    int ct4, ct6;              // CT_MAP4 / CT_MAP6 handles (-1: none)
};

// one slave entry of cilium_lb{4,6}_services (lb.h:43-81): the VIP and one backend
struct NodeService {
    uint8_t v6;
    uint8_t vip[16];           // v4: first 4 bytes
    uint8_t backend[16];
    uint16_t vport, bport;     // the key's dport and the backend's port (lb{4,6}_service.port), raw network order
};

struct NodeView {
    std::vector<NodeEndpoint> eps;
    std::vector<NodeService> svc;
    uint32_t loopback = 0;     // IPV4_LOOPBACK, raw network-order word
};

int node_view(cv_ctx *c, NodeView &v);
// what a node view depends on: the context (unique per cv_open), its endpoint generation,
// the service maps bound and their versions, the loopback address -- equal keys, equal views
struct NodeKey {
    uint64_t uid = 0, eps = 0, lb[4] = {0, 0, 0, 0}, loopback = 0;
    bool operator==(const NodeKey &o) const
    {
        return uid == o.uid && eps == o.eps && lb[0] == o.lb[0] && lb[1] == o.lb[1] && lb[2] == o.lb[2] &&
               lb[3] == o.lb[3] && loopback == o.loopback;
    }
};
int node_key(cv_ctx *c, NodeKey &k);
// live entries and max_entries of CT maps (after every batch already submitted: a sync)
int ct_counts(cv_ctx *c, const std::vector<int> &handles, std::vector<uint64_t> &live, std::vector<uint64_t> &cap);

}  // namespace cv
