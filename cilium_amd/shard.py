"""Multi-GPU partitioning of the verdict path (BASELINE config 4).

One process per GPU.  The read-only tables (prefilter, ipcache, lxc, policy, LB)
are replicated: every rank compiles them from the same agent writes.  Conntrack is
sharded: a packet belongs to the rank of its *address pair*,

    shard = mix64(min(saddr, daddr) << 32 | max(saddr, daddr)) mod world

(raw network-order words: the address pair the device groups packets by).  Every CT
entry ingress processing reads or writes -- both lookup directions, the created
tuple and its ICMP-RELATED twin, a delete -- carries the packet's address pair,
so forward, reply and related traffic meet on one rank; a 5-tuple hash would split
the related entries.  Steering packets to their owner GPU is the producer's job
(RSS-like, before the batch reaches HBM), not a collective.

The only cross-GPU data is counters: cilium_metrics (summed with one all_reduce of
the dense [256][4][2] table per reporting interval, RCCL over xGMI with the "nccl"
backend) and policy-entry packets/bytes, which the agent sums across ranks the way
it sums per-CPU map values today.
"""
from __future__ import annotations

import numpy as np

_M1, _M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)


def mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (cilium_amd/csrc/cv_common.hpp mix64)."""
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _raw32(frames: np.ndarray, off: int) -> np.ndarray:
    """the raw (little-endian load of network-order bytes) 32-bit word at `off`"""
    return np.ascontiguousarray(frames[:, off:off + 4]).view("<u4").reshape(-1)


def pair_key4(saddr_raw: np.ndarray, daddr_raw: np.ndarray) -> np.ndarray:
    lo = np.minimum(saddr_raw, daddr_raw).astype(np.uint64)
    hi = np.maximum(saddr_raw, daddr_raw).astype(np.uint64)
    return mix64((lo << np.uint64(32)) | hi)


def flow_shard(frames: np.ndarray, length: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of every IPv4 packet of a batch (non-IPv4 / short frames: rank 0,
    their verdicts touch no conntrack state on the ingress path)."""
    frames = np.asarray(frames, np.uint8)
    n = len(frames)
    out = np.zeros(n, np.int64)
    if world <= 1 or n == 0:
        return out
    eth = (frames[:, 12].astype(np.uint16) << 8) | frames[:, 13]
    v4 = (eth == 0x0800) & (np.asarray(length) >= 34)
    key = pair_key4(_raw32(frames, 26), _raw32(frames, 30))
    out[v4] = (key[v4] % np.uint64(world)).astype(np.int64)
    return out


def ct4_shard(keys: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of ipv4_ct_tuple keys (14-B rows: daddr @0, saddr @4)."""
    keys = np.asarray(keys, np.uint8)
    if world <= 1 or len(keys) == 0:
        return np.zeros(len(keys), np.int64)
    key = pair_key4(_raw32(keys, 4), _raw32(keys, 0))
    return (key % np.uint64(world)).astype(np.int64)


def split_workload(w, world: int, rank: int):
    """The rank's share of a synthetic ingress workload: its packets (in their
    original order) and its conntrack shard; the other tables stay whole."""
    import copy
    from cilium_amd import synth
    own = np.nonzero(flow_shard(w.frames, w.length, world) == rank)[0]
    maps = dict(w.maps)
    if "ct4" in maps:
        ct = maps["ct4"]
        mine = ct4_shard(ct.keys, world) == rank
        maps["ct4"] = synth.MapSpec(ct.name, ct.type, ct.key_size, ct.val_size, ct.max_entries,
                                    ct.keys[mine], ct.vals[mine])
    part = copy.copy(w)
    part.maps = maps
    part.frames = w.frames[own]
    part.length = w.length[own]
    part.mark = w.mark[own]
    return part, own


def allreduce_counters(t, group=None):
    """Sum a counter tensor (cilium_metrics [256,4,2] / policy packets, bytes) over
    all ranks: one collective per reporting interval."""
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t
