"""CPU baseline through the Linux kernel's eBPF datapath (TEST / MEASUREMENT
INFRASTRUCTURE; only bench.py's cpu_baseline leg calls it).

SURVEY.md §8(d) "CPU timing on the GPU box, same run", item (a): the hand-assembled
eBPF restatements of oracle/kernel_golden.py (config 1: bpf_xdp.c:88-184 as an XDP
program; config 2: the ingress identity + policy verdict, bpf_netdev.c:128-153,375-398
and policy.h:46-163, as a SCHED_CLS program) are loaded with the bench's full-size
tables in real kernel maps (LPM_TRIE ipcache / prefilter, HASH policy and cilium_lxc)
and run by BPF_PROG_TEST_RUN over a bounded sample of the bench's own packets, one
thread per host core, each pinned and over a disjoint slice.  Reported:

  * kernel_mpps: program runs / (the kernel-measured program time, BPF_PROG_TEST_RUN's
    `duration` x repeat, summed per thread, max over threads) — the JIT-compiled
    program with its map helpers.  Each packet runs REPEAT times in a row, so its
    lookups hit warm caches: this favours the CPU (repeat=1 adds ~4 us of test-harness
    overhead per call inside the timed region, measured on kernel 6.18);
  * harness_wall_mpps: the same runs / wall-clock, syscall + test-harness setup +
    Python included (the XDP test harness costs milliseconds per call on kernel 6.18:
    this is not a datapath figure).

Needs bpf(2) permission (root or unprivileged BPF enabled); otherwise returns the
error so bench.py can say why the figure is absent.
"""
from __future__ import annotations

import os
import struct
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
RECORDED = os.path.join(ROOT, "profiles", "cpu_kernel_ebpf.json")   # (profiles/r0*/ stay off the GPU box)
sys.path.insert(0, ROOT)

from cilium_amd import synth  # noqa: E402
from oracle import kernel_golden as K  # noqa: E402
from oracle.bpfasm import KMap, prog_load, prog_test_run, PROG_SCHED_CLS  # noqa: E402


def _load(name, w):
    """(prog fd, [maps]) for the workload's restatement program."""
    maps = []
    if name == "config1":
        km = {k: K.kmap_from_spec(v) for k, v in w.maps.items()}
        maps += list(km.values())
        v6f = KMap(synth.MAP_HASH, 20, 1, 1024)
        v6d = KMap(synth.MAP_LPM_TRIE, 20, 1, 1024, K.BPF_F_NO_PREALLOC)
        maps += [v6f, v6d]
        fd = K.xdp_prog(km["v4_dyn"], km["v4_fix"], v6d, v6f, km["lxc"])
        return fd, maps
    if name == "config2":
        ipc = K.kmap_from_spec(w.maps["ipcache"])
        pol = K.kmap_from_spec(w.maps["policy"])
        outm = KMap(2, 4, 4, 1)
        maps += [ipc, pol, outm]
        fd = prog_load(PROG_SCHED_CLS, K.policy_prog(ipc, pol, outm).assemble())
        return fd, maps
    raise ValueError(f"no eBPF restatement for {name}")


REPEAT = 32


def run(name, w, threads=None, max_packets=1 << 18, min_seconds=10.0, repeat=REPEAT):
    """Times the restatement; returns a dict for bench.py's cpu_baseline leg."""
    t0 = time.perf_counter()
    try:
        fd, maps = _load(name, w)
    except (OSError, ValueError) as e:
        try:
            sysctl = open("/proc/sys/kernel/unprivileged_bpf_disabled").read().strip()
        except OSError:
            sysctl = "?"
        out = {"error": f"{type(e).__name__}: {e} (uid {os.getuid()}, kernel.unprivileged_bpf_disabled="
                        f"{sysctl}); measured where bpf(2) is permitted: {os.path.relpath(RECORDED, ROOT)}"}
        try:                                  # the committed measurement, labelled as such
            import json
            rec = json.load(open(RECORDED))
            out["recorded_in_build_container"] = {"host": rec.get("host"), name: rec.get(name)}
        except (OSError, ValueError):
            pass
        return out
    load_s = time.perf_counter() - t0
    cpus = sorted(os.sched_getaffinity(0))
    threads = min(threads or len(cpus), len(cpus), 16)           # the GPU box's CPU share is 16
    n = min(w.n, max_packets)
    length = np.maximum(w.length[:n], 34 if name == "config2" else 14)   # test_run needs a full header
    frames = [w.frames[i, :length[i]].tobytes() for i in range(n)]
    ctxs = None
    if name == "config2":
        ctxs = []
        for i in range(n):
            c = bytearray(192)
            struct.pack_into("I", c, 8, int(w.mark[i]))
            ctxs.append(bytes(c))
    dur = [0] * threads
    cnt = [0] * threads
    err = []
    stop_at = [0.0]

    def worker(t):
        try:
            os.sched_setaffinity(0, {cpus[t]})          # this thread only (Linux TIDs)
        except OSError:
            pass
        d = c = 0
        lo, hi = t * n // threads, (t + 1) * n // threads
        try:
            i = lo
            while True:
                for _ in range(64):
                    _, ns = prog_test_run(fd, frames[i], repeat, ctxs[i] if ctxs else None)
                    d += ns * repeat
                    c += repeat
                    i = i + 1 if i + 1 < hi else lo
                if time.perf_counter() >= stop_at[0]:
                    break
        except OSError as e:
            err.append(str(e))
        dur[t], cnt[t] = d, c

    stop_at[0] = time.perf_counter() + min_seconds
    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    w0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - w0
    os.close(fd)
    for m in maps:
        m.close()
    if err:
        return {"error": err[0]}
    total = sum(cnt)
    kern_s = max(d / 1e9 for d in dur) or 1e-9
    return {"kernel_mpps": round(total / kern_s / 1e6, 3), "harness_wall_mpps": round(total / wall / 1e6, 3),
            "ns_per_packet_per_core": round(sum(dur) / total, 1), "cores": threads, "packets": total,
            "repeat": repeat,
            "sample": f"{total // repeat} calls over {n} packets of the same batch x repeat {repeat}, "
                      f"{wall:.1f} s; tables loaded in {load_s:.1f} s",
            "kernel": os.uname().release}


if __name__ == "__main__":
    wl = sys.argv[1] if len(sys.argv) > 1 else "config2"
    wk = synth.config2(1 << 16) if wl == "config2" else synth.config1(1 << 16)
    print(run(wl, wk, min_seconds=float(sys.argv[2]) if len(sys.argv) > 2 else 3.0))
