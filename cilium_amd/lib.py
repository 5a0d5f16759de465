"""ctypes binding of the product library (include/cilium_hip.h, include/cilium_agent.h,
include/cilium_epnode.h).

The library is the HIP path; there is no CPU fallback.  ``load()`` raises when
``cilium_amd/_lib/libcilium_hip.so`` is missing (build it with
``python -m cilium_amd.build``).  Batch entry points take torch CUDA (HIP) tensors
already resident in HBM and launch on torch's current stream.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CV_LIB") or os.path.join(HERE, "_lib", "libcilium_hip.so")   # CV_LIB: A/B builds
HEADER = os.path.join(os.path.dirname(HERE), "include", "cilium_hip.h")
HEADERS = [HEADER] + [os.path.join(os.path.dirname(HERE), "include", h) for h in ("cilium_agent.h", "cilium_epnode.h")]

MAP_HASH, MAP_LRU_HASH, MAP_LPM_TRIE, MAP_PERCPU_HASH = 1, 9, 11, 5
BPF_F_NO_PREALLOC = 1
ROLE_CIDR4_FIX, ROLE_CIDR4_DYN, ROLE_CIDR6_FIX, ROLE_CIDR6_DYN = 0, 1, 2, 3
ROLE_LXC, ROLE_IPCACHE, ROLE_LB4_SERVICES, ROLE_LB6_SERVICES = 4, 5, 6, 7
ROLE_LB4_REVNAT, ROLE_LB6_REVNAT = 8, 9
ROLES = {"v4_fix": 0, "v4_dyn": 1, "v6_fix": 2, "v6_dyn": 3, "lxc": 4, "ipcache": 5,
         "lb4_services": 6, "lb6_services": 7, "lb4_revnat": 8, "lb6_revnat": 9}
F_FROM_HOST, F_HAVE_L4_POLICY, F_DROP_ALL, F_CT_ACCOUNTING = 0x1, 0x2, 0x4, 0x8
F_POLICY_INGRESS, F_POLICY_EGRESS, F_DEFAULT = 0x10, 0x20, 0x3B
F_ACCT_SPLIT = 0x40              # nl / nu: conntrack lookups / writes count ACCT_CT_UNIT, the rest 1
ACCT_CT_UNIT = 32

_lib = None


class CvError(OSError):
    pass


class Batch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("stride", C.c_uint32), ("len", C.c_void_p), ("mark", C.c_void_p),
                ("n", C.c_uint32)]


OUT_FIELDS = ("xdp", "ret", "identity", "ct", "proxy", "nl", "nu", "reason", "frames_out")


class Out(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in OUT_FIELDS]


class EndpointCfg(C.Structure):
    _fields_ = [("ipv4", C.c_uint32), ("ipv6", C.c_uint8 * 16), ("mac", C.c_uint8 * 6),
                ("node_mac", C.c_uint8 * 6), ("ct6_map", C.c_int)]


class NodeCfg(C.Structure):
    _fields_ = [("ipv4_cluster_mask", C.c_uint32), ("ipv4_cluster_range", C.c_uint32),
                ("ipv4_loopback", C.c_uint32), ("router_ip6", C.c_uint8 * 16), ("host_mac", C.c_uint8 * 6),
                ("net_mac", C.c_uint8 * 6)]


def _raw_be32(v):
    """a host-order IPv4 int as the raw network-order word the C-ABI takes"""
    import struct
    return struct.unpack("<I", struct.pack(">I", v))[0]


def header_functions():
    """Names of the functions include/*.h declare."""
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(cv_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CvError(2, f"{LIB_PATH} missing: the HIP library is the product path; "
                         "build it with `python -m cilium_amd.build`")
    L = C.CDLL(LIB_PATH)
    vp, i32, u32, u64 = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64
    sig = {
        "cv_open": (i32, [i32, C.POINTER(vp)]),
        "cv_close": (None, [vp]),
        "cv_set_flags": (i32, [vp, u32]),
        "cv_version": (C.c_char_p, []),
        "cv_map_create": (i32, [vp, i32, u32, u32, u32, u32, C.POINTER(i32)]),
        "cv_map_update": (i32, [vp, i32, vp, vp, u64]),
        "cv_map_lookup": (i32, [vp, i32, vp, vp]),
        "cv_map_delete": (i32, [vp, i32, vp]),
        "cv_map_get_next_key": (i32, [vp, i32, vp, vp]),
        "cv_map_close": (i32, [vp, i32]),
        "cv_map_update_batch": (i32, [vp, i32, vp, vp, u32, u64, C.POINTER(u32)]),
        "cv_map_count": (i32, [vp, i32, C.POINTER(u32)]),
        "cv_map_dump": (i32, [vp, i32, vp, vp, u32]),
        "cv_ct_gc": (i32, [vp, i32, u32, C.POINTER(u32)]),
        "cv_ct_slots": (i32, [vp, i32, vp]),
        "cv_bind": (i32, [vp, i32, i32]),
        "cv_endpoint_add": (i32, [vp, C.c_uint16, u32, i32, i32]),
        "cv_sync": (i32, [vp]),
        "cv_publish_stats": (i32, [vp, C.POINTER(u64), C.POINTER(u64)]),
        "cv_xdp_prefilter": (i32, [vp, C.POINTER(Batch), C.POINTER(Out), vp]),
        "cv_policy_ingress": (i32, [vp, i32, C.POINTER(Batch), C.POINTER(Out), vp]),
        "cv_netdev_ingress": (i32, [vp, C.POINTER(Batch), u32, i32, C.POINTER(Out), vp]),
        "cv_lxc_egress": (i32, [vp, C.POINTER(Batch), vp, u32, vp, u32, C.POINTER(Out), vp]),
        "cv_lxc_egress_split": (i32, [vp, C.POINTER(Batch), vp, u32, vp, u32, C.POINTER(Out), vp, vp]),
        "cv_lxc_deliver": (i32, [vp, vp, u32, i32, u32, C.POINTER(Out), vp]),
        "cv_endpoint_config": (i32, [vp, i32, C.POINTER(EndpointCfg)]),
        "cv_node_config": (i32, [vp, C.POINTER(NodeCfg)]),
        "cv_metrics_read": (i32, [vp, vp]),
        "cv_metrics_reset": (i32, [vp]),
        "cv_metrics_device_ptr": (vp, [vp]),
        "cv_metrics_attach": (i32, [vp, vp]),
        "cv_notify_attach": (i32, [vp, vp, u32, vp]),
        "cv_trace_attach": (i32, [vp, vp, u32, vp, u32, u32]),
        "cv_prefilter_new": (i32, [vp, u32, C.POINTER(vp)]),
        "cv_prefilter_free": (None, [vp]),
        "cv_prefilter_insert": (i32, [vp, C.c_int64, vp, u32, C.c_char_p, u32]),
        "cv_prefilter_delete": (i32, [vp, C.c_int64, vp, u32, C.c_char_p, u32]),
        "cv_prefilter_dump": (i32, [vp, vp, u32, C.POINTER(C.c_int64)]),
        "cv_prefilter_write_config": (i32, [vp, C.c_char_p, u32]),
        "cv_prefilter_map": (i32, [vp, i32]),
        "cv_policy_sync_new": (i32, [C.POINTER(vp)]),
        "cv_policy_sync_free": (None, [vp]),
        "cv_policy_sync_set_desired": (i32, [vp, vp, vp, u32]),
        "cv_policy_sync_run": (i32, [vp, vp, i32, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]),
        "cv_policy_sync_realized": (i32, [vp, vp, vp, u32]),
        "cv_epnode_open": (i32, [vp, u32, u32, vp, u32, u32, vp, C.POINTER(vp)]),
        "cv_epnode_close": (None, [vp]),
        "cv_epnode_pending": (u64, [vp]),
        "cv_epnode_set_counts": (i32, [vp, vp, vp]),
        "cv_epnode_stats": (i32, [vp, vp]),
        "cv_epnode_sources": (i32, [vp, vp, u32]),
        "cv_epnode_sources_done": (i32, [vp, vp, vp, u32, vp, vp, vp, vp, vp, u32]),
        "cv_epnode_receive": (i32, [vp, vp, vp, vp, u32, vp]),
        "cv_epnode_deliveries": (i32, [vp, vp, vp, u32]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("CV_LIB") and not hasattr(L, name):
            continue                                   # an older A/B build without this entry point
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _lib = L
    return L


def _check(rc, what):
    if rc < 0:
        raise CvError(-rc, f"{what}: {os.strerror(-rc)}")
    return rc


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    import torch
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


# struct cv_drop_notify (include/cilium_hip.h): bpf/lib/drop.h's struct drop_notify + packet index
DROP_NOTIFY = np.dtype([("type", "u1"), ("subtype", "u1"), ("source", "<u2"), ("hash", "<u4"),
                        ("len_orig", "<u4"), ("len_cap", "<u4"), ("src_label", "<u4"), ("dst_label", "<u4"),
                        ("dst_id", "<u4"), ("ifindex", "<u4"), ("packet", "<u4"), ("reserved", "<u4")])
assert DROP_NOTIFY.itemsize == 40

# struct cv_trace_notify (include/cilium_hip.h): bpf/lib/trace.h's struct trace_notify + packet index
TRACE_NOTIFY = np.dtype([("type", "u1"), ("subtype", "u1"), ("source", "<u2"), ("hash", "<u4"),
                         ("len_orig", "<u4"), ("len_cap", "<u4"), ("src_label", "<u4"), ("dst_label", "<u4"),
                         ("dst_id", "<u2"), ("reason", "u1"), ("pad", "u1"), ("ifindex", "<u4"),
                         ("packet", "<u4"), ("reserved", "<u4")])
assert TRACE_NOTIFY.itemsize == 40
TRACE_TO_LXC, TRACE_TO_PROXY, TRACE_TO_HOST, TRACE_TO_STACK, TRACE_TO_OVERLAY = range(5)
TRACE_FROM_LXC, TRACE_FROM_PROXY, TRACE_FROM_HOST, TRACE_FROM_STACK, TRACE_FROM_OVERLAY = range(5, 10)


class Map:
    """A map handle; byte-level BPF semantics (pkg/bpf/bpf.go)."""

    def __init__(self, ctx, handle, type_, ks, vs, max_entries):
        self.ctx, self.h, self.type, self.ks, self.vs, self.max_entries = ctx, handle, type_, ks, vs, max_entries

    def update(self, key, val, flags=0):
        k, v = bytes(key), bytes(val)
        assert len(k) == self.ks and len(v) == self.vs
        return load().cv_map_update(self.ctx.h, self.h, k, v, flags)

    def update_batch(self, keys, vals, flags=0):
        keys = np.ascontiguousarray(keys, np.uint8)
        vals = np.ascontiguousarray(vals, np.uint8)
        done = C.c_uint32(0)
        rc = load().cv_map_update_batch(self.ctx.h, self.h, keys.ctypes.data, vals.ctypes.data, len(keys), flags,
                                        C.byref(done))
        _check(rc, "cv_map_update_batch")
        return done.value

    def lookup(self, key):
        v = C.create_string_buffer(self.vs)
        rc = load().cv_map_lookup(self.ctx.h, self.h, bytes(key), v)
        return (rc, v.raw if rc == 0 else None)

    def delete(self, key):
        return load().cv_map_delete(self.ctx.h, self.h, bytes(key))

    def next_key(self, key=None):
        out = C.create_string_buffer(self.ks)
        rc = load().cv_map_get_next_key(self.ctx.h, self.h, None if key is None else bytes(key), out)
        return (rc, out.raw if rc == 0 else None)

    def __len__(self):
        n = C.c_uint32(0)
        _check(load().cv_map_count(self.ctx.h, self.h, C.byref(n)), "cv_map_count")
        return n.value

    def ct_gc(self, time):
        """ctmap.GC(GCFilterByTime) (pkg/maps/ctmap/ctmap.go:325-432): delete the
        entries whose lifetime < time; time = 0xFFFFFFFF is ctmap.Flush.  Returns the
        number deleted."""
        n = C.c_uint32(0)
        _check(load().cv_ct_gc(self.ctx.h, self.h, time, C.byref(n)), "cv_ct_gc")
        return n.value

    def ct_slots(self):
        """(empty, tombstone, live) slot counts of a device CT map"""
        out = np.zeros(3, np.uint64)
        _check(load().cv_ct_slots(self.ctx.h, self.h, out.ctypes.data), "cv_ct_slots")
        return tuple(int(x) for x in out)

    def dump(self):
        n = len(self)
        keys = np.zeros((max(n, 1), self.ks), np.uint8)
        vals = np.zeros((max(n, 1), self.vs), np.uint8)
        k = _check(load().cv_map_dump(self.ctx.h, self.h, keys.ctypes.data, vals.ctypes.data, n), "cv_map_dump")
        return keys[:k], vals[:k]


class Ctx:
    """One device context (one MI355X)."""

    def __init__(self, device=0, flags=F_DEFAULT):
        L = load()
        h = C.c_void_p()
        _check(L.cv_open(device, C.byref(h)), "cv_open")
        self.h = h
        self.device = device
        if flags != F_DEFAULT:
            _check(L.cv_set_flags(self.h, flags), "cv_set_flags")

    def set_flags(self, flags):
        _check(load().cv_set_flags(self.h, flags), "cv_set_flags")

    def close(self):
        if self.h:
            load().cv_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def map_create(self, type_, ks, vs, max_entries, flags=None):
        if flags is None:
            flags = BPF_F_NO_PREALLOC if type_ == MAP_LPM_TRIE else 0
        h = C.c_int(-1)
        _check(load().cv_map_create(self.h, type_, ks, vs, max_entries, flags, C.byref(h)), "cv_map_create")
        return Map(self, h.value, type_, ks, vs, max_entries)

    def map_from_spec(self, spec):
        m = self.map_create(spec.type, spec.key_size, spec.val_size, spec.max_entries)
        m.update_batch(spec.keys, spec.vals)
        return m

    def bind(self, role, m):
        role = ROLES[role] if isinstance(role, str) else role
        _check(load().cv_bind(self.h, role, -1 if m is None else m.h), "cv_bind")

    def endpoint_add(self, lxc_id, seclabel, policy, ct4=None):
        return _check(load().cv_endpoint_add(self.h, lxc_id, seclabel, -1 if policy is None else policy.h,
                                             -1 if ct4 is None else ct4.h), "cv_endpoint_add")

    def endpoint_config(self, ep, ipv4=0, ipv6=bytes(16), mac=bytes(6), node_mac=bytes(6), ct6=None):
        """lxc_config.h constants of endpoint `ep` (ipv4 as a host-order int) and its CT_MAP6."""
        cfg = EndpointCfg(_raw_be32(ipv4), (C.c_uint8 * 16)(*bytes(ipv6)), (C.c_uint8 * 6)(*bytes(mac)),
                          (C.c_uint8 * 6)(*bytes(node_mac)), -1 if ct6 is None else ct6.h)
        _check(load().cv_endpoint_config(self.h, ep, C.byref(cfg)), "cv_endpoint_config")

    def node_config(self, cluster_mask=0, cluster_range=0, loopback=0, router_ip6=bytes(16), host_mac=bytes(6),
                    net_mac=bytes(6)):
        """node_config.h constants; the v4 words as host-order ints."""
        cfg = NodeCfg(_raw_be32(cluster_mask), _raw_be32(cluster_range), _raw_be32(loopback),
                      (C.c_uint8 * 16)(*bytes(router_ip6)), (C.c_uint8 * 6)(*bytes(host_mac)),
                      (C.c_uint8 * 6)(*bytes(net_mac)))
        _check(load().cv_node_config(self.h, C.byref(cfg)), "cv_node_config")

    def sync(self):
        _check(load().cv_sync(self.h), "cv_sync")

    def publish_stats(self):
        """(stream-ordered publications of incremental writes, table rebuilds) so far"""
        a, b = C.c_uint64(0), C.c_uint64(0)
        _check(load().cv_publish_stats(self.h, C.byref(a), C.byref(b)), "cv_publish_stats")
        return a.value, b.value

    # ---- batches (torch tensors on this device) ----
    @staticmethod
    def _batch(frames, length, mark=None):
        return Batch(frames.data_ptr(), frames.shape[1], length.data_ptr(),
                     None if mark is None else mark.data_ptr(), length.shape[0])

    @staticmethod
    def _out(o):
        o = o or {}
        return Out(*[None if o.get(k) is None else o[k].data_ptr() for k in OUT_FIELDS])

    def xdp_prefilter(self, frames, length, out):
        b, o = self._batch(frames, length), self._out(out)
        _check(load().cv_xdp_prefilter(self.h, C.byref(b), C.byref(o), _stream()), "cv_xdp_prefilter")

    def policy_ingress(self, ep, frames, length, out, mark=None):
        b, o = self._batch(frames, length, mark), self._out(out)
        _check(load().cv_policy_ingress(self.h, ep, C.byref(b), C.byref(o), _stream()), "cv_policy_ingress")

    def netdev_ingress(self, frames, length, out, now, mark=None, with_prefilter=True):
        b, o = self._batch(frames, length, mark), self._out(out)
        _check(load().cv_netdev_ingress(self.h, C.byref(b), now, 1 if with_prefilter else 0, C.byref(o), _stream()),
               "cv_netdev_ingress")

    def lxc_egress(self, frames, length, out, now, src_ep=None, flow_hash=None, ep0=0):
        b, o = self._batch(frames, length), self._out(out)
        _check(load().cv_lxc_egress(self.h, C.byref(b), _ptr(src_ep), ep0, _ptr(flow_hash), now, C.byref(o),
                                    _stream()), "cv_lxc_egress")

    def lxc_egress_split(self, frames, length, out, now, deliver, src_ep=None, flow_hash=None, ep0=0):
        """cv_lxc_egress_split: local deliveries end with ret E_DEFER (-3) and their 64-B
        record in deliver (a uint8 device tensor of n x 64)"""
        b, o = self._batch(frames, length), self._out(out)
        _check(load().cv_lxc_egress_split(self.h, C.byref(b), _ptr(src_ep), ep0, _ptr(flow_hash), now, C.byref(o),
                                          _ptr(deliver), _stream()), "cv_lxc_egress_split")

    def lxc_deliver(self, records, n, v6, out, now):
        """cv_lxc_deliver: the destination programs of n delivery records (device, n x 64 B)"""
        o = self._out(out)
        _check(load().cv_lxc_deliver(self.h, _ptr(records), n, 1 if v6 else 0, now, C.byref(o), _stream()),
               "cv_lxc_deliver")

    def metrics(self):
        m = np.zeros((256, 4, 2), np.uint64)
        _check(load().cv_metrics_read(self.h, m.ctypes.data), "cv_metrics_read")
        return m

    def metrics_reset(self):
        _check(load().cv_metrics_reset(self.h), "cv_metrics_reset")

    def metrics_attach(self, tensor):
        _check(load().cv_metrics_attach(self.h, None if tensor is None else C.c_void_p(tensor.data_ptr())),
               "cv_metrics_attach")

    def notify_attach(self, capacity):
        """Attach a device ring for drop notifications (cv_notify_attach); capacity 0
        detaches.  Returns self; read with notify_drain()."""
        import torch
        if not capacity:
            _check(load().cv_notify_attach(self.h, None, 0, None), "cv_notify_attach")
            self._notify = None
            return self
        dev = f"cuda:{self.device}"
        rec = torch.zeros(capacity * DROP_NOTIFY.itemsize, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self._notify = (rec, cnt, capacity)
        _check(load().cv_notify_attach(self.h, C.c_void_p(rec.data_ptr()), capacity, C.c_void_p(cnt.data_ptr())),
               "cv_notify_attach")
        return self

    def trace_attach(self, capacity, aggregation=0, ingress_ifindex=0):
        """Attach a device ring for trace notifications (cv_trace_attach) with the
        MONITOR_AGGREGATION level; capacity 0 detaches.  Read with trace_drain()."""
        import torch
        if not capacity:
            _check(load().cv_trace_attach(self.h, None, 0, None, 0, 0), "cv_trace_attach")
            self._trace = None
            return self
        dev = f"cuda:{self.device}"
        rec = torch.zeros(capacity * TRACE_NOTIFY.itemsize, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self._trace = (rec, cnt, capacity)
        _check(load().cv_trace_attach(self.h, C.c_void_p(rec.data_ptr()), capacity, C.c_void_p(cnt.data_ptr()),
                                      aggregation, ingress_ifindex), "cv_trace_attach")
        return self

    def trace_drain(self):
        """(records, count) of the trace ring, as notify_drain."""
        import torch
        rec, cnt, cap = self._trace
        torch.cuda.synchronize(rec.device)
        n = int(cnt.item())
        out = rec[: min(n, cap) * TRACE_NOTIFY.itemsize].cpu().numpy().view(TRACE_NOTIFY).copy()
        cnt.zero_()
        return out, n

    def notify_drain(self):
        """(records, count): the records written since the last drain (structured
        array, DROP_NOTIFY) and the number of drops (> len(records) if the ring
        overflowed); resets the ring."""
        import torch
        rec, cnt, cap = self._notify
        torch.cuda.synchronize(rec.device)
        n = int(cnt.item())
        out = rec[: min(n, cap) * DROP_NOTIFY.itemsize].cpu().numpy().view(DROP_NOTIFY).copy()
        cnt.zero_()
        return out, n


# ---------------------------------------------------------------- agent side (include/cilium_agent.h)
PF_V4_DYN, PF_V4_FIX, PF_V6_DYN, PF_V6_FIX = 0, 1, 2, 3
PF_DYN4, PF_FIX4, PF_DYN6, PF_FIX6 = 1, 2, 4, 8
PF_DEFAULT = PF_FIX4 | PF_FIX6


class Cidr(C.Structure):
    _fields_ = [("family", C.c_uint8), ("prefixlen", C.c_uint8), ("pad", C.c_uint8 * 2), ("addr", C.c_uint8 * 16)]


def cidrs_to_c(cidrs):
    """["10.0.0.0/8", "fd00::/64", ...] (net.ParseCIDR's network addresses) -> cv_cidr[]"""
    import ipaddress
    arr = (Cidr * max(len(cidrs), 1))()
    for i, c in enumerate(cidrs):
        net = ipaddress.ip_network(c, strict=False)
        arr[i].family = net.version
        arr[i].prefixlen = net.prefixlen
        raw = net.network_address.packed
        for j, b in enumerate(raw):
            arr[i].addr[j] = b
    return arr


def cidr_str(c):
    import ipaddress
    raw = bytes(c.addr[:4] if c.family == 4 else c.addr[:16])
    a = ipaddress.ip_address(raw)
    return f"{a}/{c.prefixlen}"


class PreFilter:
    """pkg/policy/prefilter.go's PreFilter over the engine (cv_prefilter_*): Insert /
    Delete raise CvError with the reference's message on failure."""

    def __init__(self, ctx, config=PF_DEFAULT):
        self.L, self.ctx = load(), ctx
        h = C.c_void_p()
        _check(self.L.cv_prefilter_new(ctx.h, config, C.byref(h)), "cv_prefilter_new")
        self.h = h

    def _op(self, fn, revision, cidrs):
        arr = cidrs_to_c(cidrs)
        err = C.create_string_buffer(512)
        rc = fn(self.h, revision, arr, len(cidrs), err, 512)
        if rc < 0:
            raise CvError(-rc, err.value.decode())

    def insert(self, revision, cidrs):
        self._op(self.L.cv_prefilter_insert, revision, cidrs)

    def delete(self, revision, cidrs):
        self._op(self.L.cv_prefilter_delete, revision, cidrs)

    def dump(self):
        rev = C.c_int64()
        n = _check(self.L.cv_prefilter_dump(self.h, None, 0, C.byref(rev)), "cv_prefilter_dump")
        arr = (Cidr * max(n, 1))()
        n = _check(self.L.cv_prefilter_dump(self.h, arr, n, C.byref(rev)), "cv_prefilter_dump")
        return [cidr_str(arr[i]) for i in range(n)], rev.value

    def write_config(self):
        n = _check(self.L.cv_prefilter_write_config(self.h, None, 0), "cv_prefilter_write_config")
        buf = C.create_string_buffer(n + 1)
        self.L.cv_prefilter_write_config(self.h, buf, n + 1)
        return buf.value.decode()

    def map_handle(self, which):
        return self.L.cv_prefilter_map(self.h, which)

    def close(self):
        if self.h:
            self.L.cv_prefilter_free(self.h)
            self.h = None


class PolicyKey(C.Structure):
    _fields_ = [("identity", C.c_uint32), ("dport", C.c_uint16), ("nexthdr", C.c_uint8), ("direction", C.c_uint8)]


class PolicySync:
    """Endpoint.syncPolicyMap's desired / realized state (cv_policy_sync_*); keys are
    (identity, dport, nexthdr, direction) in host byte order, values proxy ports."""

    def __init__(self):
        self.L = load()
        h = C.c_void_p()
        _check(self.L.cv_policy_sync_new(C.byref(h)), "cv_policy_sync_new")
        self.h = h

    def set_desired(self, desired):
        items = sorted(desired.items())
        keys = (PolicyKey * max(len(items), 1))()
        proxy = (C.c_uint16 * max(len(items), 1))()
        for i, ((ident, dport, nh, d), pp) in enumerate(items):
            keys[i] = PolicyKey(ident, dport, nh, d)
            proxy[i] = pp
        _check(self.L.cv_policy_sync_set_desired(self.h, keys, proxy, len(items)), "cv_policy_sync_set_desired")

    def run(self, ctx, policy_map):
        d, a, f = C.c_uint32(), C.c_uint32(), C.c_uint32()
        rc = self.L.cv_policy_sync_run(self.h, ctx.h, policy_map.h, C.byref(d), C.byref(a), C.byref(f))
        return rc, d.value, a.value, f.value

    def realized(self):
        n = _check(self.L.cv_policy_sync_realized(self.h, None, None, 0), "cv_policy_sync_realized")
        keys = (PolicyKey * max(n, 1))()
        proxy = (C.c_uint16 * max(n, 1))()
        n = self.L.cv_policy_sync_realized(self.h, keys, proxy, n)
        return {(k.identity, k.dport, k.nexthdr, k.direction): int(proxy[i]) for i, k in enumerate(keys[:n])}

    def close(self):
        if self.h:
            self.L.cv_policy_sync_free(self.h)
            self.h = None


# ---------------------------------------------------------------- endpoint-owned node (include/cilium_epnode.h)
class EpSched:
    """The round scheduler of one rank of the endpoint-owned node (cv_epnode_*): host
    arrays in, host arrays out; the batch, the records and the outputs stay on the
    device (cilium_amd.epnode.EpNode drives the launches)."""

    STATS = ("rounds", "source_ops", "delivery_ops", "maps_ordered_whole_at_open", "maps_ordered_whole_now",
             "rows_sent")

    def __init__(self, ctx, rank, world, frames, src_ep):
        self.L, self.world = load(), world
        frames = np.ascontiguousarray(frames, np.uint8)
        src = np.ascontiguousarray(src_ep, np.uint16)
        self.n = len(src)
        h = C.c_void_p()
        _check(self.L.cv_epnode_open(ctx.h, rank, world, frames.ctypes.data, frames.shape[1], self.n, src.ctypes.data,
                                     C.byref(h)), "cv_epnode_open")
        self.h = h
        self._pk = np.zeros(max(self.n, 1), np.uint32)

    COUNTS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int), C.c_uint32, C.POINTER(C.c_uint64),
                            C.POINTER(C.c_uint64))

    def set_counts(self, fn):
        """fn(handles) -> (live, max_entries) lists: the CT maps' counts from the caller"""
        def cb(_, hs, n, live, cap):
            try:
                lv, cp = fn([hs[i] for i in range(n)])
                for i in range(n):
                    live[i], cap[i] = int(lv[i]), int(cp[i])
                return 0
            except Exception:
                return -5
        self._cb = self.COUNTS_FN(cb)
        _check(self.L.cv_epnode_set_counts(self.h, C.cast(self._cb, C.c_void_p), None), "cv_epnode_set_counts")

    def pending(self):
        return int(self.L.cv_epnode_pending(self.h))

    def stats(self):
        a = np.zeros(6, np.uint64)
        _check(self.L.cv_epnode_stats(self.h, a.ctypes.data), "cv_epnode_stats")
        return dict(zip(self.STATS, (int(x) for x in a)))

    def sources(self):
        k = _check(self.L.cv_epnode_sources(self.h, self._pk.ctypes.data, self.n), "cv_epnode_sources")
        return self._pk[:k].copy()

    def _rows(self, cap):
        """the exchange-row buffers, reused across rounds (grown when a round needs more)"""
        if getattr(self, "_rb", None) is None or len(self._rb[0]) < cap:
            self._rb = (np.empty(cap, np.uint32), np.empty(cap, np.uint32), np.empty(cap, np.uint8),
                        np.empty(cap, np.uint32))
        return self._rb

    def sources_done(self, pkts, dst):
        """the exchange rows of the launched packets: (row_pkt, row_ep, row_has, row_pos,
        rank_rows), sorted by owner rank (views of buffers the next round reuses)"""
        pkts = np.ascontiguousarray(pkts, np.uint32)
        dst = np.ascontiguousarray(dst, np.int32)
        cap = max(2 * self.n + 64, len(self._rb[0]) if getattr(self, "_rb", None) is not None else 0)
        while True:
            rp, re_, rh, rpos = self._rows(cap)
            rr = np.zeros(self.world, np.uint32)
            k = self.L.cv_epnode_sources_done(self.h, pkts.ctypes.data, dst.ctypes.data, len(pkts), rp.ctypes.data,
                                              re_.ctypes.data, rh.ctypes.data, rpos.ctypes.data, rr.ctypes.data,
                                              len(rp))
            if k != -28:                                   # (-ENOSPC: more candidates than rows; nothing written)
                break
            cap = 4 * len(rp)
        _check(k, "cv_epnode_sources_done")
        return rp[:k], re_[:k], rh[:k], rpos[:k], rr

    def receive(self, row_pkt, row_ep, row_has):
        row_pkt = np.ascontiguousarray(row_pkt, np.uint32)
        row_ep = np.ascontiguousarray(row_ep, np.uint32)
        row_has = np.ascontiguousarray(row_has, np.uint8)
        op = np.empty(max(len(row_pkt), 1), np.int32)
        _check(self.L.cv_epnode_receive(self.h, row_pkt.ctypes.data, row_ep.ctypes.data, row_has.ctypes.data,
                                        len(row_pkt), op.ctypes.data), "cv_epnode_receive")
        return op[:len(row_pkt)]

    def deliveries(self, cap):
        if getattr(self, "_db", None) is None or len(self._db[0]) < cap:
            self._db = (np.empty(max(cap, 1), np.uint32), np.empty(max(cap, 1), np.uint32))
        ops, pk = self._db
        k = _check(self.L.cv_epnode_deliveries(self.h, ops.ctypes.data, pk.ctypes.data, cap), "cv_epnode_deliveries")
        return ops[:k].copy(), pk[:k].copy()

    def close(self):
        if self.h:
            self.L.cv_epnode_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
