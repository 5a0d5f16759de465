"""Output frames of the oracle (cv_out.frames_out): size-independent properties of
the reference's packet rewrites (lb4/lb6_xlate, reverse NAT, ipv4_l3 / ipv6_l3,
pass_to_stack's flow label), checked on CPU.

Every rewrite on the path updates the checksums incrementally (bpf_l3/l4_csum_replace
with bpf_csum_diff), so the ones-complement sum of a checksummed region, checksum field
included, must be the same before and after (mod 0xFFFF): the IPv4 header, and the
L4 segment with its pseudo header (RFC 768 / 793 / 4443).  One reference quirk breaks
the L4 sum on purpose: a service found by the L3 fallback leaves lb4/lb6_key.dport = 0,
and lb{4,6}_xlate's l4_modify_port then replaces "0" by the backend port in the
checksum while the packet's port was nonzero (lb.h:411-419, 686-694): the sum after is
the sum before minus the old port.  The arithmetic itself is
pinned by the kernel vectors (tests/golden/csum_kernel.npz, csum16_kernel.npz); this
test pins where and in which order the reference applies it."""
from __future__ import annotations

import numpy as np
import pytest

from cilium_amd import synth
from tests import harness as H


def ocsum(b: bytes) -> int:
    """ones-complement sum of 16-bit big-endian words, folded into [0, 0xFFFF)"""
    if len(b) % 2:
        b = b + b"\0"
    s = int(np.frombuffer(b, ">u2").astype(np.uint64).sum())
    return s % 0xFFFF


def l4_sum(f: bytes, v6: bool) -> int | None:
    """pseudo header (addresses, protocol) + the L4 bytes present, or None when the
    protocol has no pseudo-header checksum, an option / extension header is in the way,
    or the checksum field is not in the bytes given.  Any region holding every changed
    byte keeps its sum, so the segment need not be whole."""
    if v6:
        nh, l4 = f[20], 54
        if nh not in (6, 17, 58):
            return None
        ph = f[22:54] + bytes([0, nh])
    else:
        nh, l4 = f[23], 14 + (f[14] & 0xF) * 4
        if nh not in (6, 17) or l4 != 34:
            return None
        ph = f[26:34] + bytes([0, nh])
    coff = {6: 16, 17: 6, 58: 2}[nh]
    if l4 + coff + 2 > len(f):
        return None
    seg = f[l4:]
    if nh == 17 and seg[6:8] == b"\0\0":
        return None                                    # UDP without checksum (MARK_MANGLED_0)
    return ocsum(ph + seg)


def check_invariants(frames_in, frames_out, length, stride):
    changed = checked = quirk = 0
    for i in range(len(length)):
        a, b = bytes(frames_in[i]), bytes(frames_out[i])
        if a == b:
            continue
        changed += 1
        lim = min(int(length[i]), stride)
        a, b = a[:lim], b[:lim]
        v6 = a[12:14] == b"\x86\xdd"
        assert b[12:14] == a[12:14]
        if not v6:
            assert ocsum(a[14:34]) == ocsum(b[14:34]), i                     # IPv4 header checksum
            assert b[22] == (a[22] - 1) & 0xFF, i                            # ipv4_dec_ttl
        else:
            assert b[21] == (a[21] - 1) & 0xFF, i                            # ipv6_dec_hoplimit
            assert b[18:20] == a[18:20] and b[20] == a[20]                   # payload length, nexthdr
        sa, sb = l4_sum(a, v6), l4_sum(b, v6)
        if sa is not None:
            checked += 1
            if sa != sb:                                   # the key.dport = 0 quirk, nothing else
                l4 = 54 if v6 else 14 + (a[14] & 0xF) * 4
                old = int.from_bytes(a[l4 + 2:l4 + 4], "big")
                assert a[l4 + 2:l4 + 4] != b[l4 + 2:l4 + 4] and (sa - old) % 0xFFFF == sb, (i, v6, a.hex(), b.hex())
                quirk += 1
    return changed, checked, quirk


@pytest.mark.parametrize("family", [4, 6])
def test_config5_frame_checksums_invariant(family):
    w = synth.config5(1 << 12, n_svc=100, n_ep=32, n_remote=64, family=family, seed=81 + family)
    dp, _ = H.oracle_dp(w)
    ref = dp.lxc_egress(w.frames, w.length, w.extra["src_ep"], w.extra["flow_hash"], now=w.now, frames_out=True)
    stride = w.frames.shape[1]
    changed, checked, quirk = check_invariants(w.frames, ref.frames_out, w.length, stride)
    fwd = int(((ref.ret == 0) | (ref.ret == 7)).sum())
    assert changed > fwd // 2, (changed, fwd)
    assert checked > changed // 4, (checked, changed)
    assert quirk < checked // 4, (quirk, checked)
    if family == 6:                                     # pass_to_stack: version 6 | tclass | SECLABEL_NB
        out = ref.frames_out
        assert ((out[:, 14] >> 4)[ref.ret == 0] == 6).all()


def test_config3_frame_checksums_invariant():
    w = synth.config3(1 << 12, 1 << 10, n_ep=32, n_cidrs=512, n_ids=50, seed=13)
    dp, _ = H.oracle_dp(w)
    ref = dp.netdev_ingress(w.frames, w.length, w.mark, now=w.now, frames_out=True)
    changed, checked, quirk = check_invariants(w.frames, ref.frames_out, w.length, w.frames.shape[1])
    assert changed > 0 and checked > 0 and quirk == 0
