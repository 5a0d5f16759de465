"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker.  See cv_oracle.h for what it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libcv_oracle.so")
REF_PROBE = os.path.join(HERE, "_ref", "libref_probe.so")

F_FROM_HOST, F_HAVE_L4_POLICY, F_DROP_ALL, F_CT_ACCOUNTING = 0x1, 0x2, 0x4, 0x8
F_POLICY_INGRESS, F_POLICY_EGRESS = 0x10, 0x20
F_DEFAULT = F_FROM_HOST | F_HAVE_L4_POLICY | F_CT_ACCOUNTING | F_POLICY_INGRESS | F_POLICY_EGRESS

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE], stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        L.or_map_create.restype = vp
        L.or_map_create.argtypes = [i32, u32, u32, u32]
        L.or_map_free.argtypes = [vp]
        L.or_map_update.argtypes = [vp, vp, vp, u64]
        L.or_map_update_batch.argtypes = [vp, vp, vp, u32, u64]
        L.or_map_lookup.argtypes = [vp, vp, vp]
        L.or_map_delete.argtypes = [vp, vp]
        L.or_map_count.restype = u32
        L.or_map_count.argtypes = [vp]
        L.or_map_dump.restype = u32
        L.or_map_dump.argtypes = [vp, vp, vp, u32]
        L.or_map_digest.restype = None
        L.or_map_digest.argtypes = [vp, vp]
        L.or_set_acct_split.restype = None
        L.or_set_acct_split.argtypes = [i32]
        L.or_ct_gc.restype = u32
        L.or_ct_gc.argtypes = [vp, u32]
        L.or_get_prefix.restype = u32
        L.or_get_prefix.argtypes = [i32]
        L.or_ipv6_addr_clear_suffix.argtypes = [vp, i32]
        L.or_dp_create.restype = vp
        L.or_dp_create.argtypes = [u32]
        L.or_dp_free.argtypes = [vp]
        L.or_dp_add_endpoint.argtypes = [vp, C.c_uint16, u32, vp, vp]
        L.or_dp_metrics.argtypes = [vp, vp]
        L.or_xdp_prefilter.argtypes = [vp, vp, u32, vp, u32, vp]
        L.or_policy_ingress.argtypes = [vp, u32, vp, u32, vp, vp, u32, vp]
        L.or_netdev_ingress.argtypes = [vp, vp, u32, vp, vp, u32, u32, i32, vp]
        L.or_ct_create4.argtypes = [vp, vp, u32, i32, vp, u32]
        L.or_dp_endpoint_config.argtypes = [vp, u32, u32, vp, vp, vp, vp]
        L.or_dp_node_config.argtypes = [vp, u32, u32, u32, vp, vp, vp]
        L.or_csum_apply.argtypes = [vp, u32, u32, u32, u32, u32, u32, vp]
        L.or_lxc_egress.argtypes = [vp, vp, u32, vp, vp, u32, vp, u32, u32, vp]
        L.or_lxc_egress_split.argtypes = [vp, vp, u32, vp, vp, u32, vp, u32, u32, vp, vp, vp, vp]
        L.or_lxc_deliver.argtypes = [vp, vp, u32, vp, vp, vp, vp, vp, u32, u32, vp]
        L.or_dp_notify_attach.argtypes = [vp, vp, u32]
        L.or_dp_notify_count.restype = u32
        L.or_dp_notify_count.argtypes = [vp]
        L.or_dp_trace_attach.argtypes = [vp, vp, u32, u32, u32]
        L.or_dp_trace_count.restype = u32
        L.or_dp_trace_count.argtypes = [vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OMap:
    def __init__(self, type_, key_size, val_size, max_entries):
        self.h = lib().or_map_create(type_, key_size, val_size, max_entries)
        if not self.h:
            raise ValueError("or_map_create failed")
        self.ks, self.vs, self.max_entries = key_size, val_size, max_entries

    @classmethod
    def from_spec(cls, spec):
        m = cls(spec.type, spec.key_size, spec.val_size, spec.max_entries)
        m.load(spec.keys, spec.vals)
        return m

    def load(self, keys, vals):
        keys = np.ascontiguousarray(keys, np.uint8)
        vals = np.ascontiguousarray(vals, np.uint8)
        if len(keys):
            r = lib().or_map_update_batch(self.h, keys.ctypes.data, vals.ctypes.data, len(keys), 0)
            if r != 0:
                raise OSError(-r, "or_map_update_batch")

    def update(self, key, val, flags=0):
        k = np.ascontiguousarray(np.frombuffer(bytes(key), np.uint8))
        v = np.ascontiguousarray(np.frombuffer(bytes(val), np.uint8))
        return lib().or_map_update(self.h, k.ctypes.data, v.ctypes.data, flags)

    def lookup(self, key):
        k = np.ascontiguousarray(np.frombuffer(bytes(key), np.uint8))
        v = np.zeros(self.vs, np.uint8)
        r = lib().or_map_lookup(self.h, k.ctypes.data, v.ctypes.data)
        return (r, bytes(v) if r == 0 else None)

    def delete(self, key):
        k = np.ascontiguousarray(np.frombuffer(bytes(key), np.uint8))
        return lib().or_map_delete(self.h, k.ctypes.data)

    def ct_gc(self, time):
        """ctmap.GC (GCFilterByTime): delete CT entries with lifetime < time."""
        return lib().or_ct_gc(self.h, time)

    def __len__(self):
        return lib().or_map_count(self.h)

    def dump(self):
        n = len(self)
        keys = np.zeros((max(n, 1), self.ks), np.uint8)
        vals = np.zeros((max(n, 1), self.vs), np.uint8)
        k = lib().or_map_dump(self.h, _p(keys), _p(vals), n)
        return keys[:k], vals[:k]

    def digest(self):
        """(count, sum, xor) of the per-entry chains (tests/harness.table_digest)"""
        out = np.zeros(3, np.uint64)
        lib().or_map_digest(self.h, out.ctypes.data)
        return tuple(int(x) for x in out)

    def __del__(self):
        try:
            lib().or_map_free(self.h)
        except Exception:
            pass


class Out:
    """Per-packet oracle outputs (SoA)."""

    def __init__(self, n):
        self.xdp = np.zeros(n, np.uint8)
        self.ret = np.zeros(n, np.int32)
        self.identity = np.zeros(n, np.uint32)
        self.ct = np.zeros(n, np.uint8)
        self.proxy = np.zeros(n, np.uint16)
        self.nl = np.zeros(n, np.uint8)
        self.nu = np.zeros(n, np.uint8)
        self.reason = np.zeros(n, np.int32)

    FIELDS = ("xdp", "ret", "identity", "ct", "proxy", "nl", "nu", "reason")
    frames_out = None          # set to an (n, stride) uint8 array to receive the rewritten frames

    def struct(self):
        ptrs = [getattr(self, k).ctypes.data for k in self.FIELDS]
        ptrs.append(None if self.frames_out is None else self.frames_out.ctypes.data)
        return (C.c_void_p * 9)(*ptrs)


class ODp:
    """The oracle datapath: maps bound by role, endpoints, metrics."""

    ROLES = ("v4_fix", "v4_dyn", "v6_fix", "v6_dyn", "lxc", "ipcache", "lb4_services", "lb6_services",
             "lb4_revnat", "lb6_revnat")

    def __init__(self, flags=F_DEFAULT):
        self.h = lib().or_dp_create(flags)
        self.maps = {}
        self.keep = []

    def bind(self, role, omap):
        idx = self.ROLES.index(role)
        # or_dp layout: the role map pointers first, in ROLES order
        ptrs = C.cast(self.h, C.POINTER(C.c_void_p))
        ptrs[idx] = omap.h
        self.maps[role] = omap

    def add_endpoint(self, lxc_id, seclabel, policy, ct4=None):
        self.keep += [policy, ct4]
        return lib().or_dp_add_endpoint(self.h, lxc_id, seclabel, policy.h if policy is not None else None,
                                        ct4.h if ct4 is not None else None)

    def endpoint_config(self, ep, ipv4=0, ipv6=None, mac=None, node_mac=None, ct6=None):
        """lxc_config.h constants of endpoint `ep` (ipv4 as a host-order int) and its CT_MAP6."""
        import struct
        raw4 = struct.unpack("<I", struct.pack(">I", ipv4))[0]
        bufs = [None if b is None else C.create_string_buffer(bytes(b), len(bytes(b))) for b in (ipv6, mac, node_mac)]
        if ct6 is not None:
            self.keep.append(ct6)
        r = lib().or_dp_endpoint_config(self.h, ep, raw4, *bufs, ct6.h if ct6 is not None else None)
        if r:
            raise OSError(-r, "or_dp_endpoint_config")

    def node_config(self, cluster_mask=0, cluster_range=0, loopback=0, router_ip6=b"\0" * 16, host_mac=b"\0" * 6,
                    net_mac=b"\0" * 6):
        """node_config.h constants; the v4 words as host-order ints (written in network order)."""
        import struct
        raw = [struct.unpack("<I", struct.pack(">I", v))[0] for v in (cluster_mask, cluster_range, loopback)]
        lib().or_dp_node_config(self.h, *raw, C.create_string_buffer(bytes(router_ip6), 16),
                                C.create_string_buffer(bytes(host_mac), 6), C.create_string_buffer(bytes(net_mac), 6))

    def notify_attach(self, capacity):
        """Record drop notifications (send_drop_notify) into a host ring."""
        from cilium_amd.lib import DROP_NOTIFY
        self._nbuf = np.zeros(max(capacity, 1), DROP_NOTIFY)
        self._ncap = capacity
        lib().or_dp_notify_attach(self.h, self._nbuf.ctypes.data if capacity else None, capacity)

    def trace_attach(self, capacity, aggregation=0, ingress_ifindex=0):
        """Record trace notifications (send_trace_notify) into a host ring."""
        from cilium_amd.lib import TRACE_NOTIFY
        self._tbuf = np.zeros(max(capacity, 1), TRACE_NOTIFY)
        self._tcfg = (capacity, aggregation, ingress_ifindex)
        lib().or_dp_trace_attach(self.h, self._tbuf.ctypes.data if capacity else None, capacity, aggregation,
                                 ingress_ifindex)

    def trace_drain(self):
        n = lib().or_dp_trace_count(self.h)
        out = self._tbuf[: min(n, self._tcfg[0])].copy()
        lib().or_dp_trace_attach(self.h, self._tbuf.ctypes.data, *self._tcfg)
        return out, n

    def notify_drain(self):
        n = lib().or_dp_notify_count(self.h)
        out = self._nbuf[: min(n, self._ncap)].copy()
        lib().or_dp_notify_attach(self.h, self._nbuf.ctypes.data, self._ncap)
        return out, n

    def metrics(self):
        m = np.zeros((256, 4, 2), np.uint64)
        lib().or_dp_metrics(self.h, m.ctypes.data)
        return m

    def lxc_egress(self, frames, length, src_ep=None, flow_hash=None, now=0, ep0=0, frames_out=False):
        n = len(length)
        out = Out(n)
        if frames_out:
            out.frames_out = np.zeros(np.asarray(frames).shape, np.uint8)
        frames = np.ascontiguousarray(frames, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        src_ep = None if src_ep is None else np.ascontiguousarray(src_ep, np.uint16)
        flow_hash = None if flow_hash is None else np.ascontiguousarray(flow_hash, np.uint32)
        s = out.struct()
        lib().or_lxc_egress(self.h, _p(frames), frames.shape[1], _p(length), _p(src_ep), ep0, _p(flow_hash), n,
                            now, C.byref(s))
        return out

    def lxc_egress_split(self, frames, length, src_ep, flow_hash, now=0):
        """lxc_egress stopped at local deliveries (ret OR_E_DEFER = -3): returns the outputs
        (frames_out holds the frames as the source programs left them) and, per packet,
        the destination endpoint index (-1: none), its ifindex and the source seclabel."""
        n = len(length)
        out = Out(n)
        frames = np.ascontiguousarray(frames, np.uint8)
        out.frames_out = np.zeros(frames.shape, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        src_ep = np.ascontiguousarray(src_ep, np.uint16)
        flow_hash = np.ascontiguousarray(flow_hash, np.uint32)
        dl = np.full(n, -1, np.int32)
        ifx = np.zeros(n, np.uint32)
        lab = np.zeros(n, np.uint32)
        s = out.struct()
        lib().or_lxc_egress_split(self.h, _p(frames), frames.shape[1], _p(length), _p(src_ep), 0, _p(flow_hash), n,
                                  now, C.byref(s), _p(dl), _p(ifx), _p(lab))
        return out, dl, ifx, lab

    def lxc_deliver(self, frames, length, dl_ep, dl_ifindex, dl_label, nl, nu, now=0):
        """the destination programs of deferred packets (nl / nu: the source programs' counts)"""
        n = len(length)
        out = Out(n)
        out.nl[:] = nl
        out.nu[:] = nu
        frames = np.ascontiguousarray(frames, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        args = [np.ascontiguousarray(a, t) for a, t in ((dl_ep, np.int32), (dl_ifindex, np.uint32),
                                                         (dl_label, np.uint32))]
        s = out.struct()
        lib().or_lxc_deliver(self.h, _p(frames), frames.shape[1], _p(length), *[_p(a) for a in args], None, n, now,
                             C.byref(s))
        return out

    def xdp_prefilter(self, frames, length):
        n = len(length)
        out = Out(n)
        frames = np.ascontiguousarray(frames, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        s = out.struct()
        lib().or_xdp_prefilter(self.h, _p(frames), frames.shape[1], _p(length), n, C.byref(s))
        return out

    def policy_ingress(self, ep_index, frames, length, mark=None):
        n = len(length)
        out = Out(n)
        frames = np.ascontiguousarray(frames, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        mark = None if mark is None else np.ascontiguousarray(mark, np.uint32)
        s = out.struct()
        lib().or_policy_ingress(self.h, ep_index, _p(frames), frames.shape[1], _p(length), _p(mark), n,
                                C.byref(s))
        return out

    def netdev_ingress(self, frames, length, mark=None, now=0, with_prefilter=True, frames_out=False):
        n = len(length)
        out = Out(n)
        if frames_out:
            out.frames_out = np.zeros(np.asarray(frames).shape, np.uint8)
        frames = np.ascontiguousarray(frames, np.uint8)
        length = np.ascontiguousarray(length, np.uint32)
        mark = None if mark is None else np.ascontiguousarray(mark, np.uint32)
        s = out.struct()
        lib().or_netdev_ingress(self.h, _p(frames), frames.shape[1], _p(length), _p(mark), n, now,
                                1 if with_prefilter else 0, C.byref(s))
        return out

    def __del__(self):
        try:
            lib().or_dp_free(self.h)
        except Exception:
            pass


def csum_apply(frame, op, off, frm, to, flags):
    """The oracle's restatement of the kernel checksum helpers on one frame (bytes):
    returns (rc, frame after, csum_diff result)."""
    b = np.frombuffer(bytes(frame), np.uint8).copy()
    d = C.c_uint64(0)
    rc = lib().or_csum_apply(b.ctypes.data, len(b), op, off, frm, to, flags, C.byref(d))
    return rc, bytes(b), d.value


def ref_probe():
    """The reference's own pure helpers (oracle/_ref), or None if not built."""
    if not os.path.exists(REF_PROBE):
        return None
    L = C.CDLL(REF_PROBE)
    L.ref_get_prefix.restype = C.c_uint32
    L.ref_get_prefix.argtypes = [C.c_int]
    L.ref_ipv6_addr_clear_suffix.argtypes = [C.c_void_p, C.c_int]
    L.ref_layout.restype = C.c_long
    L.ref_layout.argtypes = [C.c_int]
    return L


def set_acct_split(on):
    """nl / nu count conntrack lookups / writes 32 each (include/cilium_hip.h CV_F_ACCT_SPLIT)"""
    lib().or_set_acct_split(1 if on else 0)
