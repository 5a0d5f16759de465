"""Golden vectors from the Linux kernel itself (TEST INFRASTRUCTURE).

Runs in the build container (root, bpf(2) available) and writes small fixtures to
tests/golden/.  Three pins for the oracle:

  * kernel map semantics: the same update/delete/lookup sequences on real kernel
    HASH and LPM_TRIE maps (kernel/bpf/hashtab.c, lpm_trie.c) -> return codes and
    lookup results;
  * config 1: a hand-assembled eBPF restatement of bpf/bpf_xdp.c (check_filters /
    check_v4 / check_v6 / check_v{4,6}_endpoint, :88-184) run by BPF_PROG_TEST_RUN
    over synthetic frames with real kernel LPM + HASH + cilium_lxc maps;
  * config 2: a hand-assembled SCHED_CLS restatement of the ingress verdict
    (bpf_netdev.c:128-153 identity from mark, :375-398 ipcache resolution,
    conntrack.h:471-530 L4 key of a NEW flow, policy.h:46-163 policy with
    __sync_fetch_and_add counters) by BPF_PROG_TEST_RUN with skb->mark in ctx_in.

Usage: python -m oracle.kernel_golden   (from the repo root)
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from cilium_amd import synth  # noqa: E402
from oracle.bpfasm import (Asm, KMap, insn, prog_load, prog_test_run, PROG_XDP, PROG_SCHED_CLS,  # noqa: E402
                           BPF_F_NO_PREALLOC, R0, R1, R2, R3, R4, R5, R6, R7, R8, R9, FP)

GOLDEN = os.path.join(ROOT, "tests", "golden")
MAP_LOOKUP = 1


def kmap_from_spec(spec):
    flags = BPF_F_NO_PREALLOC if spec.type == synth.MAP_LPM_TRIE else 0
    m = KMap(spec.type, spec.key_size, spec.val_size, spec.max_entries, flags)
    for k, v in zip(spec.keys, spec.vals):
        r = m.update(k.tobytes(), v.tobytes())
        if r:
            raise OSError(-r, "kernel map update")
    return m


# ------------------------------------------------------------------------
# bpf_xdp.c restatement
# ------------------------------------------------------------------------

def xdp_prog(v4_dyn, v4_fix, v6_dyn, v6_fix, lxc):
    a = Asm()
    a.mov(R6, R1)
    a.ldxw(R7, R6, 0)                  # xdp->data
    a.ldxw(R8, R6, 4)                  # xdp->data_end
    a.mov(R2, R7); a.addi(R2, 14); a.jgt(R2, R8, "drop")      # xdp_no_room(eth + 1)
    a.ldxh(R3, R7, 12)
    a.jeqi(R3, 0x0008, "v4")           # bpf_htons(ETH_P_IP)
    a.jeqi(R3, 0xDD86, "v6")           # bpf_htons(ETH_P_IPV6)
    a.ja("pass")
    # check_v4 (:97-121)
    a.label("v4")
    a.mov(R2, R7); a.addi(R2, 34); a.jgt(R2, R8, "drop")
    a.stw(FP, -8, 32)
    a.ldxw(R3, R7, 26); a.stxw(FP, -4, R3)
    if v4_dyn is not None:
        a.ld_map(R1, v4_dyn.fd); a.mov(R2, FP); a.addi(R2, -8); a.call(MAP_LOOKUP)
        a.jnei(R0, 0, "drop")
    if v4_fix is not None:
        a.ld_map(R1, v4_fix.fd); a.mov(R2, FP); a.addi(R2, -8); a.call(MAP_LOOKUP)
        a.jnei(R0, 0, "drop")
    # check_v4_endpoint (:88-95) -> lookup_ip4_endpoint (eps.h:37-46)
    a.stdw(FP, -32, 0); a.stdw(FP, -24, 0); a.stw(FP, -16, 0)
    a.ldxw(R3, R7, 30); a.stxw(FP, -32, R3)
    a.stb(FP, -16, 1)
    a.ld_map(R1, lxc.fd); a.mov(R2, FP); a.addi(R2, -32); a.call(MAP_LOOKUP)
    a.jnei(R0, 0, "pass")
    a.ja("drop")
    # check_v6 (:132-156)
    a.label("v6")
    a.mov(R2, R7); a.addi(R2, 54); a.jgt(R2, R8, "drop")
    a.stw(FP, -24, 128)
    for i in range(4):
        a.ldxw(R3, R7, 22 + 4 * i); a.stxw(FP, -20 + 4 * i, R3)
    if v6_dyn is not None:
        a.ld_map(R1, v6_dyn.fd); a.mov(R2, FP); a.addi(R2, -24); a.call(MAP_LOOKUP)
        a.jnei(R0, 0, "drop")
    if v6_fix is not None:
        a.ld_map(R1, v6_fix.fd); a.mov(R2, FP); a.addi(R2, -24); a.call(MAP_LOOKUP)
        a.jnei(R0, 0, "drop")
    a.stdw(FP, -48, 0); a.stdw(FP, -40, 0); a.stw(FP, -32, 0)
    for i in range(4):
        a.ldxw(R3, R7, 38 + 4 * i); a.stxw(FP, -48 + 4 * i, R3)
    a.stb(FP, -32, 2)
    a.ld_map(R1, lxc.fd); a.mov(R2, FP); a.addi(R2, -48); a.call(MAP_LOOKUP)
    a.jnei(R0, 0, "pass")
    a.label("drop"); a.movi(R0, 1); a.exit()          # XDP_DROP
    a.label("pass"); a.movi(R0, 2); a.exit()          # XDP_PASS
    return prog_load(PROG_XDP, a.assemble())


def v6_frames(saddr16, daddr16, n, stride=64):
    f = np.zeros((n, stride), np.uint8)
    f[:, 12:14] = [0x86, 0xDD]
    f[:, 14] = 0x60
    f[:, 20] = 6
    f[:, 21] = 64
    f[:, 22:38] = saddr16
    f[:, 38:54] = daddr16
    return f


def gen_config1(n=16384):
    w = synth.config1(n)
    s = synth.Stream(0xC1A0F001)
    # IPv6 prefilter tables + frames (v6 maps sized with the v4 ELEMS, bpf_xdp.c:73,83)
    n6 = 64
    v6_fix = s.u64(n6 * 2).view(np.uint8).reshape(n6, 16)
    v6_dyn_len = s.randint(n6, 16, 128)
    v6_dyn = s.u64(n6 * 2).view(np.uint8).reshape(n6, 16).copy()
    for i in range(n6):
        b = bytearray(v6_dyn[i].tobytes())
        for bit in range(int(v6_dyn_len[i]), 128):
            b[bit // 8] &= ~(0x80 >> (bit % 8)) & 0xFF
        v6_dyn[i] = np.frombuffer(bytes(b), np.uint8)
    lxc6 = s.u64(32 * 2).view(np.uint8).reshape(32, 16)

    def v6key(addr, plen):
        k = np.zeros((len(addr), 20), np.uint8)
        k[:, 0:4] = synth.le32_bytes(np.asarray(plen, np.uint32))
        k[:, 4:20] = addr
        return k
    maps = dict(w.maps)
    maps["v6_fix"] = synth.MapSpec("cilium_cidr_v6_fix", synth.MAP_HASH, 20, 1, 1 << 20,
                                   v6key(v6_fix, np.full(n6, 128)), np.zeros((n6, 1), np.uint8))
    maps["v6_dyn"] = synth.MapSpec("cilium_cidr_v6_dyn", synth.MAP_LPM_TRIE, 20, 1, 1 << 16,
                                   v6key(v6_dyn, v6_dyn_len), np.zeros((n6, 1), np.uint8))
    lk = np.zeros((32, 20), np.uint8); lk[:, 0:16] = lxc6; lk[:, 16] = 2
    lx = maps["lxc"]
    maps["lxc"] = synth.MapSpec(lx.name, lx.type, 20, 48, lx.max_entries,
                                np.concatenate([lx.keys, lk]),
                                np.concatenate([lx.vals, synth.endpoint_infos(np.arange(32), np.arange(5000, 5032),
                                                                              np.zeros(32))]))
    m6 = 1024
    r = s.frac(m6)
    sa = np.where((r < 0.3)[:, None], v6_fix[s.choice(m6, n6)],
                  np.where((r < 0.6)[:, None], v6_dyn[s.choice(m6, n6)], s.u64(m6 * 2).view(np.uint8).reshape(m6, 16)))
    da = np.where((s.frac(m6) < 0.7)[:, None], lxc6[s.choice(m6, 32)], s.u64(m6 * 2).view(np.uint8).reshape(m6, 16))
    f6 = v6_frames(sa, da, m6)
    l6 = np.full(m6, 64, np.uint32)
    l6[:32] = s.randint(32, 14, 54)                     # short v6 frames
    frames = np.concatenate([w.frames, f6])
    length = np.concatenate([w.length, l6])
    length = np.maximum(length, 14)                      # test_run needs >= ETH_HLEN

    km = {k: kmap_from_spec(v) for k, v in maps.items()}
    fd = xdp_prog(km["v4_dyn"], km["v4_fix"], km["v6_dyn"], km["v6_fix"], km["lxc"])
    verdict = np.zeros(len(length), np.uint8)
    for i in range(len(length)):
        verdict[i], _ = prog_test_run(fd, frames[i, :length[i]].tobytes())
    os.close(fd)
    for m in km.values():
        m.close()
    out = {"frames": frames, "length": length, "verdict": verdict}
    for name, sp in maps.items():
        out[f"map_{name}_keys"] = sp.keys
        out[f"map_{name}_vals"] = sp.vals
        out[f"map_{name}_meta"] = np.array([sp.type, sp.key_size, sp.val_size, sp.max_entries])
    np.savez_compressed(os.path.join(GOLDEN, "c1_xdp_kernel.npz"), **out)
    print("config1 xdp:", len(length), "frames", np.bincount(verdict))


# ------------------------------------------------------------------------
# config 2: identity + policy verdict restatement (SCHED_CLS)
# ------------------------------------------------------------------------

def policy_prog(ipcache, policy, outmap):
    a = Asm()
    a.mov(R6, R1)
    a.ldxw(R7, R6, 76)                 # skb->data
    a.ldxw(R8, R6, 80)                 # skb->data_end
    # identity from mark (handle_identity_from_host, bpf_netdev.c:128-153); r9 = identity
    a.ldxw(R3, R6, 8)                  # skb->mark
    a.mov(R4, R3); a.andi(R4, 0xF00)
    a.stdw(FP, -56, 0)                 # fp-56: skip_proxy flag
    a.movi(R9, 2)                      # WORLD_ID
    a.jeqi(R4, 0xC00, "id_host")
    a.jeqi(R4, 0xA00, "id_proxy_in")
    a.jeqi(R4, 0xB00, "id_proxy")
    a.ja("id_done")
    a.label("id_host"); a.movi(R9, 1); a.ja("id_done")
    a.label("id_proxy_in"); a.stdw(FP, -56, 1)
    a.label("id_proxy")
    a.mov(R9, R3); a.andi(R9, 0xFF); a.lshi(R9, 16)
    a.mov(R4, R3); a.rshi(R4, 16); a.orr(R9, R4)   # (mark & 0xFF) << 16 | mark >> 16
    a.label("id_done")
    a.stxw(FP, -20, R9)                # fp-20: resolved identity (output)
    # L3 checks
    a.mov(R2, R7); a.addi(R2, 14); a.jgt(R2, R8, "unknown_l3")
    a.ldxh(R3, R7, 12); a.jnei(R3, 0x0008, "unknown_l3")
    a.mov(R2, R7); a.addi(R2, 34); a.jgt(R2, R8, "invalid")
    # ipcache resolution for reserved identities (bpf_netdev.c:375-398)
    a.jgei(R9, 4, "l4")
    a.stdw(FP, -48, 0); a.stdw(FP, -40, 0); a.stdw(FP, -32, 0)
    a.stw(FP, -48, 64); a.stb(FP, -41, 1)
    a.ldxw(R3, R7, 26); a.stxw(FP, -40, R3)
    a.ld_map(R1, ipcache.fd); a.mov(R2, FP); a.addi(R2, -48); a.call(MAP_LOOKUP)
    a.jeqi(R0, 0, "l4")
    a.ldxw(R3, R0, 0)
    a.jeqi(R3, 0, "l4"); a.jeqi(R3, 3, "l4"); a.jeqi(R3, 1, "l4")
    a.mov(R9, R3)
    a.stxw(FP, -20, R9)
    # L4 key of a NEW flow (conntrack.h:471-530, after the tuple reverse)
    a.label("l4")
    a.stxw(FP, -8, R9)                 # policy_key.sec_label (identity)
    a.ldxb(R4, R7, 23)                 # nexthdr
    a.ldxb(R3, R7, 14); a.andi(R3, 0xF); a.lshi(R3, 2); a.addi(R3, 14)  # l4_off
    a.mov(R1, R7)
    a.emit(insn(0x0f, R1, R3))         # r1 = data + l4_off (variable-offset packet pointer)
    a.jeqi(R4, 6, "tcp")
    a.jeqi(R4, 17, "udp")
    a.jeqi(R4, 1, "icmp")
    a.movi(R0, -137); a.ja("out")      # DROP_CT_UNKNOWN_PROTO
    a.label("tcp")
    a.mov(R2, R1); a.addi(R2, 14); a.jgt(R2, R8, "badhdr")
    a.ldxh(R3, R1, 2); a.ja("key")
    a.label("udp")
    a.mov(R2, R1); a.addi(R2, 4); a.jgt(R2, R8, "badhdr")
    a.ldxh(R3, R1, 2); a.ja("key")
    a.label("icmp")
    a.mov(R2, R1); a.addi(R2, 1); a.jgt(R2, R8, "badhdr")
    a.ldxb(R3, R1, 0)
    a.jeqi(R3, 8, "key")               # ECHO: sport = type -> dport after reverse = 8
    a.movi(R3, 0)
    a.label("key")
    a.stxh(FP, -4, R3); a.stxb(FP, -2, R4); a.stb(FP, -1, 0)
    a.stxw(FP, -12, R3)                # save dport
    a.stxw(FP, -16, R4)                # save proto
    a.ldxw(R9, R6, 0)                  # skb->len
    # __policy_can_access (policy.h:51-119), HAVE_L4_POLICY
    a.ld_map(R1, policy.fd); a.mov(R2, FP); a.addi(R2, -8); a.call(MAP_LOOKUP)
    a.jnei(R0, 0, "hit_l4")
    a.sth(FP, -4, 0); a.stb(FP, -2, 0)
    a.ld_map(R1, policy.fd); a.mov(R2, FP); a.addi(R2, -8); a.call(MAP_LOOKUP)
    a.jnei(R0, 0, "hit_l3")
    a.stw(FP, -8, 0)
    a.ldxw(R3, FP, -12); a.stxh(FP, -4, R3)
    a.ldxw(R4, FP, -16); a.stxb(FP, -2, R4)
    a.ld_map(R1, policy.fd); a.mov(R2, FP); a.addi(R2, -8); a.call(MAP_LOOKUP)
    a.jnei(R0, 0, "hit_l4")
    a.movi(R0, -133); a.ja("out")      # DROP_POLICY
    a.label("hit_l3")
    a.movi(R3, 1); a.emit(insn(0xdb, R0, R3, 8)); a.emit(insn(0xdb, R0, R9, 16))
    a.movi(R0, 0); a.ja("out")
    a.label("hit_l4")
    a.movi(R3, 1); a.emit(insn(0xdb, R0, R3, 8)); a.emit(insn(0xdb, R0, R9, 16))
    a.ldxh(R0, R0, 0)                  # proxy_port (raw be16)
    a.ldxdw(R3, FP, -56)
    a.jeqi(R3, 0, "out")
    a.movi(R0, 0); a.ja("out")         # skip_proxy -> verdict 0
    a.label("unknown_l3"); a.movi(R0, -139); a.ja("out")
    a.label("invalid"); a.movi(R0, -134); a.ja("out")
    a.label("badhdr"); a.movi(R0, -135); a.ja("out")
    # out: store identity in outmap[0], return r0
    a.label("out")
    a.stxw(FP, -28, R0)                # keep ret
    a.stw(FP, -32, 0)
    a.ld_map(R1, outmap.fd); a.mov(R2, FP); a.addi(R2, -32); a.call(MAP_LOOKUP)
    a.jeqi(R0, 0, "ret")
    a.ldxw(R3, FP, -20); a.stxw(R0, 0, R3)
    a.label("ret")
    a.ldxw(R0, FP, -28)
    a.exit()
    return a


def gen_config2(n=8192):
    w = synth.config2(n, n_cidrs=4096, n_ids=500)
    s = synth.Stream(0xC1A0F002)
    mark = np.zeros(n, np.uint32)
    sel = s.frac(n) < 0.05
    mark[sel] = (s.u32(int(sel.sum())) & np.uint32(0xFFFF00FF)) | np.uint32(0xC00)
    sel2 = s.frac(n) < 0.05
    mark[sel2] = (np.uint32(400) << 16 | np.uint32(0xA00)) if sel2.any() else 0
    length = w.length.copy()
    short = s.frac(n) < 0.01
    length[short] = s.randint(int(short.sum()), 34, 48).astype(np.uint32)  # skb test_run needs a full iphdr
    ipc = kmap_from_spec(w.maps["ipcache"])
    pol = kmap_from_spec(w.maps["policy"])
    outm = KMap(2, 4, 4, 1)            # BPF_MAP_TYPE_ARRAY
    a = policy_prog(ipc, pol, outm)
    fd = prog_load(PROG_SCHED_CLS, a.assemble())
    ret = np.zeros(n, np.int32)
    ident = np.zeros(n, np.uint32)
    for i in range(n):
        ctx = bytearray(192)
        struct.pack_into("I", ctx, 8, int(mark[i]))
        rv, _ = prog_test_run(fd, w.frames[i, :length[i]].tobytes(), ctx=bytes(ctx))
        ret[i] = np.int32(np.uint32(rv).view(np.int32))
        ident[i] = struct.unpack("I", outm.lookup(b"\0\0\0\0")[1])[0]
    counters = np.zeros((len(w.maps["policy"].keys), 24), np.uint8)
    for i, k in enumerate(w.maps["policy"].keys):
        r, v = pol.lookup(k.tobytes())
        counters[i] = np.frombuffer(v, np.uint8)
    os.close(fd)
    for m in (ipc, pol, outm):
        m.close()
    out = {"frames": w.frames, "length": length, "mark": mark, "ret": ret, "identity": ident,
           "policy_vals_after": counters}
    for name, sp in w.maps.items():
        out[f"map_{name}_keys"] = sp.keys
        out[f"map_{name}_vals"] = sp.vals
        out[f"map_{name}_meta"] = np.array([sp.type, sp.key_size, sp.val_size, sp.max_entries])
    np.savez_compressed(os.path.join(GOLDEN, "c2_policy_kernel.npz"), **out)
    vals, cnt = np.unique(ret, return_counts=True)
    print("config2 policy:", n, "packets", dict(zip(vals.tolist()[:8], cnt.tolist()[:8])), "...")


# ------------------------------------------------------------------------
# map semantics sequences
# ------------------------------------------------------------------------

def gen_map_semantics():
    s = synth.Stream(0xC1A0F003)
    cases = []
    # HASH 8->4, max 64; LPM 8->4 (v4) and 24->8 (ipcache-shaped), max 64
    for (typ, ks, vs, mx) in [(1, 8, 4, 64), (11, 8, 4, 64), (11, 24, 8, 128)]:
        km = KMap(typ, ks, vs, mx, BPF_F_NO_PREALLOC if typ == 11 else 0)
        ops = []
        pool = []
        for i in range(600):
            r = float(s.frac(1)[0])
            if r < 0.55 or not pool:
                if typ == 11:
                    k = bytearray(s.u64(4).view(np.uint8)[:ks].tobytes())
                    plen = int(s.randint(1, 0, (ks - 4) * 8 + 3)[0])   # occasionally invalid (> max)
                    if ks == 24 and float(s.frac(1)[0]) < 0.7:
                        plen = 32 + int(s.randint(1, 0, 33)[0])
                        k[4:8] = b"\0\0\0\1"
                        k[12:24] = b"\0" * 12
                    k[0:4] = struct.pack("I", plen)
                    k = bytes(k)
                else:
                    k = s.u64(1).view(np.uint8).tobytes()
                    k = k[:4] + bytes([k[4] & 3, 0, 0, 0])
                v = s.u64(2).view(np.uint8)[:vs].tobytes()
                fl = int(s.randint(1, 0, 4)[0])
                rc = km.update(k, v, fl)
                ops.append((0, k, v, fl, rc))
                if rc == 0:
                    pool.append(k)
            elif r < 0.75:
                k = pool[int(s.choice(1, len(pool))[0])]
                rc = km.delete(k)
                ops.append((1, k, b"\0" * vs, 0, rc))
            else:
                k = bytearray(pool[int(s.choice(1, len(pool))[0])])
                if typ == 11:   # lookup: full-length key with random host bits
                    k[0:4] = struct.pack("I", (ks - 4) * 8 if ks == 8 else 64)
                    if float(s.frac(1)[0]) < 0.5:
                        k[len(k) - 1] ^= int(s.randint(1, 0, 256)[0])
                rc, v = km.lookup(bytes(k))
                ops.append((2, bytes(k), v if v else b"\0" * vs, 0, rc))
        km.close()
        cases.append(((typ, ks, vs, mx), ops))
    out = {}
    for ci, ((typ, ks, vs, mx), ops) in enumerate(cases):
        out[f"c{ci}_meta"] = np.array([typ, ks, vs, mx])
        out[f"c{ci}_op"] = np.array([o[0] for o in ops], np.int32)
        out[f"c{ci}_key"] = np.array([np.frombuffer(o[1], np.uint8) for o in ops])
        out[f"c{ci}_val"] = np.array([np.frombuffer(o[2], np.uint8) for o in ops])
        out[f"c{ci}_flags"] = np.array([o[3] for o in ops], np.int32)
        out[f"c{ci}_rc"] = np.array([o[4] for o in ops], np.int32)
    out["ncases"] = np.array(len(cases))
    np.savez_compressed(os.path.join(GOLDEN, "map_semantics_kernel.npz"), **out)
    print("map semantics:", [len(c[1]) for c in cases], "ops")


# ------------------------------------------------------------------------
# checksum helpers: bpf_l3_csum_replace / bpf_l4_csum_replace / bpf_csum_diff
# (net/core/filter.c on the container's kernel), the arithmetic of every packet
# rewrite on the path (lb.h lb4_xlate / __lb4_rev_nat, l3.h ipv4_l3 -> ipv4_dec_ttl)
# ------------------------------------------------------------------------
CSUM_FRAME = 96          # eth + ipv4 + tcp, params @64, csum_diff result @84
H_STORE, H_L3, H_L4, H_LOAD, H_DIFF = 9, 10, 11, 26, 28


def csum_prog():
    """op = u32 @64: 0 l3_csum_replace(skb, off, from, to, flags), 1 l4_csum_replace,
    2 csum_diff(&from, 4, &to, 4, seed) -> u64 stored @84; params off/from/to/flags
    (seed) as u32 @68/@72/@76/@80."""
    a = Asm()
    a.mov(R6, R1)
    a.mov(R1, R6); a.movi(R2, 64); a.mov(R3, FP); a.addi(R3, -32); a.movi(R4, 20); a.call(H_LOAD)
    a.jnei(R0, 0, "out")
    a.ldxw(R7, FP, -32)
    a.ldxw(R2, FP, -28); a.ldxw(R3, FP, -24); a.ldxw(R4, FP, -20); a.ldxw(R5, FP, -16)
    a.jeqi(R7, 0, "l3")
    a.jeqi(R7, 1, "l4")
    a.mov(R1, FP); a.addi(R1, -24); a.movi(R2, 4); a.mov(R3, FP); a.addi(R3, -20); a.movi(R4, 4)
    a.call(H_DIFF)
    a.stxw(FP, -8, R0)
    a.rshi(R0, 32)
    a.stxw(FP, -4, R0)
    a.mov(R1, R6); a.movi(R2, 84); a.mov(R3, FP); a.addi(R3, -8); a.movi(R4, 8); a.movi(R5, 0); a.call(H_STORE)
    a.ja("out")
    a.label("l3"); a.mov(R1, R6); a.call(H_L3); a.ja("out")
    a.label("l4"); a.mov(R1, R6); a.call(H_L4)
    a.label("out"); a.movi(R0, 0); a.exit()
    return a


def gen_csum(n=6000):
    from oracle.bpfasm import prog_test_run_out
    s = synth.Stream(0xC1A0F004)
    fd = prog_load(PROG_SCHED_CLS, csum_prog().assemble())
    base = synth.ipv4_frames(np.array([0x0A000001], np.uint32), np.array([0x0A000002], np.uint32),
                             np.array([6], np.uint8), np.array([1234]), np.array([80]), np.array([0x10]),
                             np.array([64]))[0]
    fin = np.zeros((n, CSUM_FRAME), np.uint8)
    fout = np.zeros((n, CSUM_FRAME), np.uint8)
    edge = np.array([0x0000, 0xFFFF, 0x0001, 0xFFFE, 0x8000, 0x7FFF], np.uint32)
    for i in range(n):
        f = np.zeros(CSUM_FRAME, np.uint8)
        f[:64] = base
        op = int(s.choice(1, 3)[0])
        r = s.u32(6)
        ck = int(edge[r[0] % len(edge)]) if r[1] % 4 == 0 else int(r[2] & 0xFFFF)
        if op == 0:
            off, size = 24, int([0, 2, 4][r[3] % 3])
            flags = size
        elif op == 1:
            udp = r[3] % 2 == 1
            off = 40 if udp else 50
            f[23] = 17 if udp else 6
            size = int([0, 2, 4][(r[3] >> 1) % 3])
            flags = size | (0x10 if (r[3] >> 3) & 1 else 0) | (0x20 if udp and (r[3] >> 4) & 1 else 0)
            if udp and (r[3] >> 5) % 4 == 0:
                ck = 0                                    # UDP without checksum
        else:
            off, flags = 0, int(edge[r[4] % len(edge)] * 0x10001) if r[5] % 4 == 0 else int(r[4])
        frm, to = int(r[4]), int(r[5])
        if op != 2 and (flags & 0xF) == 2:
            frm, to = frm & 0xFFFF, to & 0xFFFF
        if op != 2 and (flags & 0xF) == 0:
            frm = 0
        if op != 2:
            f[off:off + 2] = np.frombuffer(struct.pack(">H", ck), np.uint8)
        f[64:84] = np.frombuffer(struct.pack("<IIIII", op, off, frm, to, flags & 0xFFFFFFFF), np.uint8)
        _, out = prog_test_run_out(fd, f.tobytes())
        fin[i] = f
        fout[i] = np.frombuffer(out[:CSUM_FRAME], np.uint8)
    os.close(fd)
    np.savez_compressed(os.path.join(GOLDEN, "csum_kernel.npz"), frames_in=fin, frames_out=fout)
    print("csum helpers:", n, "cases;", int((fin != fout).any(axis=1).sum()), "changed frames")


CSUM16_FRAME = 112       # from16 @64, to16 @80, seed @96, csum_diff result @104


def csum16_prog():
    """csum_diff(from16, 16, to16, 16, seed) -> u64 stored @104: the sum of the IPv6
    address rewrites (lb6_xlate lb.h:405, __lb6_rev_nat lb.h:289)."""
    a = Asm()
    a.mov(R6, R1)
    a.mov(R1, R6); a.movi(R2, 64); a.mov(R3, FP); a.addi(R3, -48); a.movi(R4, 36); a.call(H_LOAD)
    a.jnei(R0, 0, "out")
    a.ldxw(R5, FP, -16)
    a.mov(R1, FP); a.addi(R1, -48); a.movi(R2, 16); a.mov(R3, FP); a.addi(R3, -32); a.movi(R4, 16)
    a.call(H_DIFF)
    a.stxw(FP, -8, R0)
    a.rshi(R0, 32)
    a.stxw(FP, -4, R0)
    a.mov(R1, R6); a.movi(R2, 104); a.mov(R3, FP); a.addi(R3, -8); a.movi(R4, 8); a.movi(R5, 0); a.call(H_STORE)
    a.label("out"); a.movi(R0, 0); a.exit()
    return a


def gen_csum16(n=4000):
    """Golden vectors of the 16-byte bpf_csum_diff: random addresses and seeds, plus
    edge words (all-zero, all-ones, equal from/to, single-bit differences)."""
    from oracle.bpfasm import prog_test_run_out
    s = synth.Stream(0xC1A0F016)
    fd = prog_load(PROG_SCHED_CLS, csum16_prog().assemble())
    fin = np.zeros((n, CSUM16_FRAME), np.uint8)
    fout = np.zeros((n, CSUM16_FRAME), np.uint8)
    edge = np.array([0, 0xFFFFFFFF, 1, 0xFFFF, 0xFFFF0000, 0x80000000], np.uint32)
    for i in range(n):
        f = np.zeros(CSUM16_FRAME, np.uint8)
        f[12:14] = (0x86, 0xDD)
        r = s.u32(12)
        words = r[:8].copy()
        kind = int(r[8] % 6)
        if kind == 1:
            words[:] = edge[r[9] % len(edge)]
        elif kind == 2:
            words[4:] = words[:4]                                  # from == to
        elif kind == 3:
            words[4:] = words[:4] ^ np.uint32(1 << int(r[9] % 32))   # one bit differs
        elif kind == 4:
            words[:4] = edge[r[9] % len(edge)]
            words[4:] = edge[r[10] % len(edge)]
        seed = int(edge[r[11] % len(edge)]) if r[10] % 4 == 0 else int(r[11])
        f[64:100] = np.frombuffer(struct.pack("<8I", *[int(w) for w in words]) + struct.pack("<I", seed), np.uint8)
        _, out = prog_test_run_out(fd, f.tobytes())
        fin[i] = f
        fout[i] = np.frombuffer(out[:CSUM16_FRAME], np.uint8)
    os.close(fd)
    np.savez_compressed(os.path.join(GOLDEN, "csum16_kernel.npz"), frames_in=fin, frames_out=fout)
    print("csum_diff 16:", n, "cases")


if __name__ == "__main__":
    os.makedirs(GOLDEN, exist_ok=True)
    which = sys.argv[1:] or ["maps", "config1", "config2", "csum", "csum16"]
    if "csum16" in which:
        gen_csum16()
    if "maps" in which:
        gen_map_semantics()
    if "config1" in which:
        gen_config1()
    if "config2" in which:
        gen_config2()
    if "csum" in which:
        gen_csum()
