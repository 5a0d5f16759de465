"""Minimal eBPF assembler + bpf(2) syscall wrappers (TEST INFRASTRUCTURE).

Used only to generate golden vectors in the build container (root, kernel bpf
available): real kernel maps (kernel/bpf/hashtab.c, lpm_trie.c) and
BPF_PROG_TEST_RUN of hand-assembled restatements of the reference's BPF programs.
Follows the loading pattern of the reference's bpf/probes/raw_main.c
(BPF_PROG_LOAD of instruction arrays with map-fd fixups); written fresh.
"""
from __future__ import annotations

import ctypes as C
import os
import struct

SYS_bpf = 321
BPF_MAP_CREATE, BPF_MAP_LOOKUP_ELEM, BPF_MAP_UPDATE_ELEM, BPF_MAP_DELETE_ELEM = 0, 1, 2, 3
BPF_MAP_GET_NEXT_KEY, BPF_PROG_LOAD, BPF_PROG_TEST_RUN = 4, 5, 10
PROG_XDP, PROG_SCHED_CLS = 6, 3
BPF_F_NO_PREALLOC = 1

_libc = C.CDLL(None, use_errno=True)


def _bpf(cmd, attr: bytes):
    buf = C.create_string_buffer(attr + b"\0" * (144 - len(attr)), 144)
    r = _libc.syscall(SYS_bpf, cmd, buf, 144)
    if r < 0:
        return -C.get_errno(), buf
    return r, buf


class KMap:
    def __init__(self, type_, ks, vs, max_entries, flags=0):
        r, _ = _bpf(BPF_MAP_CREATE, struct.pack("IIIII", type_, ks, vs, max_entries, flags))
        if r < 0:
            raise OSError(-r, "BPF_MAP_CREATE")
        self.fd, self.ks, self.vs = r, ks, vs

    def update(self, key: bytes, val: bytes, flags=0) -> int:
        kb, vb = C.create_string_buffer(key, self.ks), C.create_string_buffer(val, self.vs)
        r, _ = _bpf(BPF_MAP_UPDATE_ELEM, struct.pack("IIQQQ", self.fd, 0, C.addressof(kb), C.addressof(vb), flags))
        return 0 if r >= 0 else r

    def lookup(self, key: bytes):
        kb, vb = C.create_string_buffer(key, self.ks), C.create_string_buffer(self.vs)
        r, _ = _bpf(BPF_MAP_LOOKUP_ELEM, struct.pack("IIQQQ", self.fd, 0, C.addressof(kb), C.addressof(vb), 0))
        return (0, vb.raw[:self.vs]) if r >= 0 else (r, None)

    def delete(self, key: bytes) -> int:
        kb = C.create_string_buffer(key, self.ks)
        r, _ = _bpf(BPF_MAP_DELETE_ELEM, struct.pack("IIQ", self.fd, 0, C.addressof(kb)))
        return 0 if r >= 0 else r

    def close(self):
        os.close(self.fd)


# ---- instruction encoding (include/uapi/linux/bpf.h, bpf_common.h) ----
R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, FP = range(11)


def insn(op, dst=0, src=0, off=0, imm=0):
    return struct.pack("<BBhi", op, (src << 4) | dst, off, imm)


class Asm:
    def __init__(self):
        self.code = []          # list of (bytes | label-fixup tuple)
        self.labels = {}

    def label(self, name):
        self.labels[name] = len(self.code)

    def emit(self, b):
        self.code.append(b)

    # ALU64
    def mov(self, d, s):   self.emit(insn(0xbf, d, s))
    def movi(self, d, k):  self.emit(insn(0xb7, d, 0, 0, k))
    def addi(self, d, k):  self.emit(insn(0x07, d, 0, 0, k))
    def andi(self, d, k):  self.emit(insn(0x57, d, 0, 0, k))
    def rshi(self, d, k):  self.emit(insn(0x77, d, 0, 0, k))
    def lshi(self, d, k):  self.emit(insn(0x67, d, 0, 0, k))
    def orr(self, d, s):   self.emit(insn(0x4f, d, s))
    # memory
    def ldxw(self, d, s, off):  self.emit(insn(0x61, d, s, off))
    def ldxh(self, d, s, off):  self.emit(insn(0x69, d, s, off))
    def ldxb(self, d, s, off):  self.emit(insn(0x71, d, s, off))
    def ldxdw(self, d, s, off): self.emit(insn(0x79, d, s, off))
    def stxw(self, d, off, s):  self.emit(insn(0x63, d, s, off))
    def stxh(self, d, off, s):  self.emit(insn(0x6b, d, s, off))
    def stxb(self, d, off, s):  self.emit(insn(0x73, d, s, off))
    def stxdw(self, d, off, s): self.emit(insn(0x7b, d, s, off))
    def stw(self, d, off, k):   self.emit(insn(0x62, d, 0, off, k))
    def sth(self, d, off, k):   self.emit(insn(0x6a, d, 0, off, k))
    def stb(self, d, off, k):   self.emit(insn(0x72, d, 0, off, k))
    def stdw(self, d, off, k):  self.emit(insn(0x7a, d, 0, off, k))

    def ld_map(self, d, fd):
        self.emit(insn(0x18, d, 1, 0, fd))       # BPF_PSEUDO_MAP_FD
        self.emit(insn(0x00, 0, 0, 0, 0))

    def call(self, helper): self.emit(insn(0x85, 0, 0, 0, helper))
    def exit(self):          self.emit(insn(0x95))

    # jumps with label fixups
    def _j(self, op, d, s, k, lbl):
        self.code.append(("J", op, d, s, k, lbl))

    def ja(self, lbl):              self._j(0x05, 0, 0, 0, lbl)
    def jeqi(self, d, k, lbl):      self._j(0x15, d, 0, k, lbl)
    def jnei(self, d, k, lbl):      self._j(0x55, d, 0, k, lbl)
    def jgti(self, d, k, lbl):      self._j(0x25, d, 0, k, lbl)
    def jgei(self, d, k, lbl):      self._j(0x35, d, 0, k, lbl)
    def jlti(self, d, k, lbl):      self._j(0xa5, d, 0, k, lbl)
    def jgt(self, d, s, lbl):       self._j(0x2d, d, s, 0, lbl)
    def jeq(self, d, s, lbl):       self._j(0x1d, d, s, 0, lbl)
    def jne(self, d, s, lbl):       self._j(0x5d, d, s, 0, lbl)

    def assemble(self) -> bytes:
        out = []
        for i, c in enumerate(self.code):
            if isinstance(c, tuple):
                _, op, d, s, k, lbl = c
                out.append(insn(op, d, s, self.labels[lbl] - i - 1, k))
            else:
                out.append(c)
        return b"".join(out)


def prog_load(prog_type, code: bytes, license_=b"GPL"):
    lic = C.create_string_buffer(license_)
    ib = C.create_string_buffer(code, len(code))
    log = C.create_string_buffer(1 << 16)
    attr = struct.pack("IIQQIIQ", prog_type, len(code) // 8, C.addressof(ib), C.addressof(lic), 1,
                       1 << 16, C.addressof(log))
    r, _ = _bpf(BPF_PROG_LOAD, attr)
    if r < 0:
        raise OSError(-r, "BPF_PROG_LOAD: " + log.value.decode(errors="replace")[-2000:])
    return r


def prog_test_run(fd, data: bytes, repeat=1, ctx: bytes | None = None):
    """Returns (retval, duration_ns)."""
    db = C.create_string_buffer(data, len(data))
    cb = C.create_string_buffer(ctx, len(ctx)) if ctx else None
    attr = struct.pack("IIIIQQII IIQQ".replace(" ", ""), fd, 0, len(data), 0, C.addressof(db), 0, repeat, 0,
                       len(ctx) if ctx else 0, 0, C.addressof(cb) if cb else 0, 0)
    r, buf = _bpf(BPF_PROG_TEST_RUN, attr)
    if r < 0:
        raise OSError(-r, "BPF_PROG_TEST_RUN")
    _, retval, _, _, _, _, _, duration = struct.unpack_from("IIIIQQII", buf.raw)
    return retval, duration


def prog_test_run_out(fd, data: bytes, ctx: bytes | None = None):
    """BPF_PROG_TEST_RUN returning (retval, data_out): the packet after the program
    (skb programs get a CHECKSUM_NONE skb)."""
    db = C.create_string_buffer(data, len(data))
    ob = C.create_string_buffer(len(data) + 256)
    cb = C.create_string_buffer(ctx, len(ctx)) if ctx else None
    attr = struct.pack("IIIIQQIIIIQQ", fd, 0, len(data), len(data) + 256, C.addressof(db), C.addressof(ob), 1, 0,
                       len(ctx) if ctx else 0, 0, C.addressof(cb) if cb else 0, 0)
    r, buf = _bpf(BPF_PROG_TEST_RUN, attr)
    if r < 0:
        raise OSError(-r, "BPF_PROG_TEST_RUN")
    _, retval, _, size_out = struct.unpack_from("IIII", buf.raw)
    return retval, ob.raw[:size_out]
