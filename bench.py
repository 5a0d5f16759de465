#!/usr/bin/env python3
"""Benchmark of the MI355X batch verdict engine (BASELINE.json metric).

A step = one pass of the verdict path over one batch of synthetic packets already
resident in HBM.  Default workload = config 3, the largest single-GPU 64-B config:
the full bpf_lxc ingress path (XDP prefilter -> from_netdev -> handle_ipv4 ->
endpoint ipv4_policy with conntrack) over 2^24 64-B IPv4 headers per step against a
16M-flow conntrack table, on one MI355X per rank.  --workload config1 / config2 /
config4 / config5 measure the other paths.

Stateful workloads (conntrack: configs 3, 4, 5) give every step its own batch: step v
is the batch with fresh client ports on its new flows (synth.port_variant), so every
timed step creates the conntrack entries the workload's new flows need instead of
replaying flows an earlier pass created.  The batches are built on the device before
the timed region; the CT tables are sized for every create of the run.  The
accounting pass (L(p), U(p) of SURVEY.md §8(d)) is one more such step after the
timed region.

Multi-GPU (torchrun): tables are replicated, every rank verdicts its own batch
(weak scaling, no data-path collective); conntrack is sharded by address pair
(cilium_amd.shard): at N > 1 configs 3 / 4 give each rank 16M flows of one node-wide
flow set (128M on 8 GPUs) and packets of its own pairs; cilium_metrics is summed
across ranks with one RCCL all_reduce after the timed region.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "Mpps verdicts at 1/2/4/8 GPUs (64B hdrs); achieved HBM GB/s vs peak"

WORKLOADS = {
    "config3": "full bpf_lxc ingress path: prefilter + ipcache + lxc + policy + ct_lookup4/ct_create4, 16M-flow CT "
               "per GPU (at N > 1 one node-wide flow set sharded by address pair = config 4), "
               "a fresh batch per step (20% new flows)",
    "config2": "ipcache LPM (100k CIDRs->identities) + policymap (10k identities x L4 ports) ingress verdicts",
    "config1": "bpf_xdp.c CIDR deny-list prefilter, 1k IPv4 prefixes + cilium_lxc",
    "config4": "config 3 per GPU with conntrack sharded by address pair (16M flows per GPU, 128M on 8), "
               "RCCL all_reduce of cilium_metrics",
    "config5": "dual-stack from-container egress: lb4/lb6 (50k services) + CT4/CT6 + egress policy + local delivery "
               "(v4 64-B and v6 128-B records, 1:1), a fresh batch per step (20% of flows new)",
}
STATEFUL = ("config3", "config4", "config5")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def lib_sha():
    """the device code the PMC summaries were taken with (cilium_amd/build.py kernel_sha)"""
    from cilium_amd import build
    return build.kernel_sha()


def make_workload(name, n, rank, world, flows=1 << 24, zipf=None, ep_zipf=None):
    from cilium_amd import synth
    if name == "config2":
        return synth.config2(n)
    if name == "config1":
        return synth.config1(n)
    if name in ("config3", "config4"):
        # N > 1: the rank's part of one node-wide flow set (16M flows per rank), the flows
        # whose address pair it owns, and packets of its own pairs (pre-steered by the
        # producer): conntrack sharded by address pair, config 4 of BASELINE.json
        seed = 0xC1A00003 if name == "config3" else 0xC1A00004
        return synth.config3(n, n_flows=flows, seed=seed, shard=(rank, world) if world > 1 else None, zipf=zipf,
                             ep_zipf=ep_zipf)
    if name == "config5":
        return synth.config5(n, ep_zipf=ep_zipf)
    raise SystemExit(f"unknown workload {name}")


def size_conntrack(name, w, passes):
    """max_entries of the CT maps for a run of `passes` fresh batches: today's entries
    plus every create the run can make (config 3: the tuple and its RELATED twin per
    new-flow packet; config 5: up to 7 entries per fresh flow over the families), with
    room, as a power of two."""
    def p2(x):
        return 1 << int(np.ceil(np.log2(max(x, 1 << 16))))
    if name in ("config3", "config4"):
        nn = int((w.extra["kind"] == 2).sum())
        ct = w.maps["ct4"]
        ct.max_entries = p2((len(ct.keys) + 2 * nn * (passes + 1)) * 1.2)
    elif name == "config5":
        for fam in ("ct4", "ct6"):
            w.maps[fam].max_entries = p2(0.9 * w.n + 0.45 * w.n * passes)


def split_families(w):
    """config 5: the v4 packets as 64-B records and the v6 packets as 128-B records
    (two launches per step; v4 and v6 state are disjoint, so order between them is free).
    Returns the parts and, per packet of w, (part index, row in part)."""
    v6 = w.extra["v6"]
    parts, where = [], np.zeros((w.n, 2), np.int64)
    for k, (sel, stride) in enumerate(((~v6, 64), (v6, 128))):
        idx = np.nonzero(sel)[0]
        where[idx, 0] = k
        where[idx, 1] = np.arange(len(idx))
        parts.append({"frames": np.ascontiguousarray(w.frames[idx, :stride]), "length": w.length[idx],
                      "src_ep": w.extra["src_ep"][idx], "flow_hash": w.extra["flow_hash"][idx]})
    return parts, where


def to_device(a, device):
    """a host array on the device (u16 / u32 as the int16 / int32 views torch holds)"""
    import torch
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def step_batch(name, w, v, base, where, device):
    """Step v's batch, built on the device from the resident base batch: the workload with
    fresh client ports on its new flows (synth.port_variant).  Config 5: the two family
    parts (base = their device frames, where = split_families' row map); else one frame
    array."""
    import torch
    from cilium_amd import synth
    rows, boff, ports = synth.port_variant(w, v)
    hi = torch.from_numpy((ports >> 8).astype(np.uint8)).to(device)
    lo = torch.from_numpy((ports & 0xFF).astype(np.uint8)).to(device)
    if name == "config5":
        fv = [p.clone() for p in base]
        for k in (0, 1):
            sel = where[rows, 0] == k
            r = torch.from_numpy(where[rows[sel], 1]).to(device)
            o = torch.from_numpy(boff[sel]).to(device)
            s = torch.from_numpy(sel).to(device)
            fv[k][r, o] = hi[s]
            fv[k][r, o + 1] = lo[s]
        return fv
    fv = base.clone()
    r, o = torch.from_numpy(rows).to(device), torch.from_numpy(boff).to(device)
    fv[r, o] = hi
    fv[r, o + 1] = lo
    return fv


def algorithmic_bytes(name, nl, nu, record=64):
    """B(p) = R + V + 64*L(p) + 64*U(p), summed over the batch."""
    R = record
    V = {"config1": 4, "config2": 8, "config3": 9, "config4": 9, "config5": 9}[name]
    n = len(nl)
    return n * (R + V) + 64 * (int(nl.astype(np.int64).sum()) + int(nu.astype(np.int64).sum()))


def hbm_resident_bytes(ct, ret, record=64, V=9):
    """config 3: the algorithmic bytes of the HBM-resident part -- the record stream, the
    outputs and the conntrack lines (a 2^27..2^28-entry table) -- from each packet's CT
    result as ct_lookup4 (conntrack.h:442-562) reaches it: REPLY / RELATED one probe,
    ESTABLISHED / NEW two (the tuple, then its reverse); a hit writes its line back; an
    allowed NEW writes the tuple and its ICMP twin.  The rest of B(p) (policy, ipcache,
    endpoint and prefilter lines) stays in L2 / Infinity Cache."""
    ct = ct.astype(np.int64)
    lines = np.where((ct == 2) | (ct == 3), 1, np.where((ct == 0) | (ct == 1), 2, 0))
    lines += np.where((ct >= 1) & (ct <= 3), 1, 0)
    lines += np.where((ct == 0) & ((ret == 0) | (ret == 7)), 2, 0)       # TC_ACT_OK / TC_ACT_REDIRECT
    return len(ct) * (record + V) + 64 * int(lines.sum())


def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    share = cpu_share()
    return {"cpu_model": model, "nproc": os.cpu_count(), "kernel": platform.release(), **share}


_OMP_ENV = os.environ.get("OMP_NUM_THREADS")


def cpu_share():
    """The host CPUs this process may use: its affinity mask, the cgroup CPU quota
    (cpu.max) and the lease's OMP_NUM_THREADS, whichever is smallest.  nproc counts the
    whole machine; a GPU lease grants a share of it."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    env = int(_OMP_ENV) if _OMP_ENV and _OMP_ENV.isdigit() else None
    use = min(x for x in (aff, quota, env) if x)
    return {"cpus_affinity": aff, "cpus_cgroup_quota": quota, "omp_num_threads_env": env, "threads_used": use}


def allowed_cpus():
    return cpu_share()["threads_used"]


def cpu_baseline(name, w, min_seconds=10.0):
    """The oracle (plain-C restatement) timed on the host cores on a bounded sample of
    the same workload (>= min_seconds of CPU work).  Stateless paths (configs 1, 2):
    OpenMP over the threads.  Conntrack ingress (configs 3, 4): the sample partitioned
    by address pair over the threads, one oracle datapath per shard with its CT shard
    (tests/harness.ShardedOracle; identical results to one sequential run).  Egress
    (config 5): one replica per thread (tables replicated, each with its own
    conntrack), the way bench.py runs that path on N GPUs.  Stateful samples are re-run as fresh
    steps (synth.port_variant), as on the GPU."""
    from cilium_amd import synth
    from tests import harness as H
    threads = allowed_cpus()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    done, busy, v = 0, 0.0, 0
    if name in ("config1", "config2"):
        sample = min(w.n, 1 << 21)
        dp, _ = H.oracle_dp(w)
        frames, length, mark = w.frames[:sample], w.length[:sample], w.mark[:sample]
        run = (lambda: dp.xdp_prefilter(frames, length)) if name == "config1" else \
              (lambda: dp.policy_ingress(0, frames, length, mark))
        while busy < min_seconds:
            t0 = time.perf_counter()
            run()
            busy += time.perf_counter() - t0
            done += sample
        cores, how = threads, f"OpenMP {threads} threads"
    else:
        import copy
        from concurrent.futures import ThreadPoolExecutor
        sample = min(w.n, 1 << 20 if name != "config5" else 1 << 18)
        sw = copy.copy(w)
        sw.frames, sw.length, sw.mark = w.frames[:sample], w.length[:sample], w.mark[:sample]
        sw.extra = {k: (x[:sample] if isinstance(x, np.ndarray) and len(x) == w.n else x) for k, x in w.extra.items()
                    if not isinstance(k, tuple)}                  # (not port_variant's cache of the full batch)
        if name == "config5":
            # one replica per thread (tables replicated, each its own conntrack and its
            # own fresh batches), as bench.py runs the GPUs for this path at N > 1
            pool = ThreadPoolExecutor(threads)
            dps = list(pool.map(lambda _: H.oracle_dp(sw)[0], range(threads)))
            cores, how = threads, f"{threads} threads, one replica (tables + own conntrack) each"
            while busy < min_seconds:
                v += 1
                fs = [H.apply_variant(sw.frames, *synth.port_variant(sw, v))] * threads
                t0 = time.perf_counter()
                list(pool.map(lambda t: dps[t].lxc_egress(fs[t], sw.length, sw.extra["src_ep"], sw.extra["flow_hash"],
                                                          now=w.now + v), range(threads)))
                busy += time.perf_counter() - t0
                done += sample * threads
            pool.shutdown()
        else:
            so = H.ShardedOracle(sw, threads)
            pool = ThreadPoolExecutor(threads)
            cores, how = threads, f"{threads} threads, one address-pair CT shard each"
            while busy < min_seconds:
                v += 1
                f = H.apply_variant(sw.frames, *synth.port_variant(sw, v))
                _, el = so.netdev_ingress(f, now=w.now + v, pool=pool)
                busy += el
                done += sample
            pool.shutdown()
    return {"value": round(done / busy / 1e6, 3), "unit": "Mpps", "cores": cores, "kind": "port",
            "sample": f"oracle/cv_oracle.c over {done} packets of the synthetic {name} batch ({v or 1} "
                      f"step{'s' if v > 1 else ''} of {done // max(v, 1)}; {busy:.1f} s; {how})",
            "host": dict(host_info(), threads_used=cores)}


def random_access_peak():
    """SURVEY.md §8(d) denominator 1, measured in this run: random 64-B line reads
    (4 x dwordx4 per lane) from a 4 GiB table in HBM (tools/gather_probe.hip, built by
    __graft_entry__.build()), best of 3 launches of 2^26 reads; GB/s of whole lines."""
    import ctypes as C
    so = os.path.join(ROOT, "tools", "libgather_probe.so")
    if not os.path.exists(so):
        return None
    L = C.CDLL(so)
    L.probe_run.restype = C.c_float
    L.probe_run.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_int, C.c_int]
    n = 1 << 26
    ms = L.probe_run(0, 4 << 30, n, 8192, 3)
    return None if ms <= 0 else round(n * 64 / (ms * 1e-3) / 1e9, 1)


def pmc_traffic(name, sha):
    """HBM bytes per step from the committed rocprofv3 --pmc summary of this exact
    device code (profiles/pmc_<workload>.json, keyed by build.kernel_sha), else None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
    except Exception:
        return None
    if d.get("kernel_sha") != sha:
        return None
    return d.get("hbm_bytes_per_step", d.get("hbm_bytes_per_launch"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="config3", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg and the random-access probe (profiling runs)")
    ap.add_argument("--ct-room", type=int, default=None,
                    help="max_entries = the preloaded entries + this many (0: a full table, every "
                         "create fails; the exact-admission regime) instead of room for every create of the run")
    ap.add_argument("--ct-max-log2", type=int, default=None,
                    help="max_entries = 2^N (the device table: 2^N entries at 60%% slot load) instead "
                         "of room for every create of the run; with --gc-step the run stays within it")
    ap.add_argument("--ct-max", type=int, default=None,
                    help="max_entries of every CT map (config 5: CT4 and CT6; a run that creates more fills them "
                         "and then runs next to the limit: the exact-admission regime)")
    ap.add_argument("--gc-step", type=int, default=0,
                    help="steady state: every step is this many seconds after the previous one and ctmap.GC "
                         "(cv_ct_gc, GCFilterByTime at the step's now) runs before it, inside the timed region")
    ap.add_argument("--flows", type=int, default=1 << 24, help="configs 3/4: conntrack flows per GPU")
    ap.add_argument("--zipf", type=float, default=None,
                    help="configs 3/4: Zipf(a) flow popularity for the existing flows' packets (elephant flows)")
    ap.add_argument("--ct-local", type=int, default=None,
                    help="configs 3/4/5: ConntrackLocal -- every endpoint its own CT4 map (config 5: CT4 and CT6) "
                         "of this max_entries (ctmap.go:54: 64000) holding its flows' preloaded entries "
                         "(synth.per_endpoint_ct)")
    ap.add_argument("--ep-zipf", type=float, default=None,
                    help="configs 3/4: Zipf(a) popularity of the endpoints the preloaded flows belong to; config 5: "
                         "of the flows' client endpoints (with --ct-local: the busiest endpoints' maps are full)")
    ap.add_argument("--ep-owned", action="store_true",
                    help="config 5 as ONE node across the ranks with endpoint-owned conntrack (cilium_amd.epnode, "
                         "include/cilium_epnode.h): every endpoint its own CT4 / CT6 map (--ct-local, default 64000), "
                         "rank r runs the source programs of the endpoints e %% N == r and the deliveries into them, "
                         "records exchanged per round (RCCL all_to_all); every rank holds the whole batch "
                         "(--packets, default 2^20) and the node processes it once per step")
    ap.add_argument("--dist-backend", default="nccl", help="torch.distributed backend at N > 1 (nccl = RCCL)")
    ap.add_argument("--dump", default=None,
                    help="test hook: every rank writes <dir>/rank<r>.npz (its packets' address-pair keys, its "
                         "cilium_metrics before and after the all_reduce)")
    args = ap.parse_args()

    # the JSON line is the only thing on stdout: everything else (libraries that print
    # to fd 1, e.g. gloo's connection messages) goes to stderr
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
    device = f"cuda:{local}"
    torch.cuda.set_device(local)

    from cilium_amd import build as cvbuild
    from cilium_amd import synth
    cvbuild.build()
    from tests import harness as H

    if args.ep_owned:
        return ep_owned(args, rank, world, local, device, dist, out_fd)
    name = args.workload
    stateful = name in STATEFUL
    passes = args.warmup + args.steps + 1                          # + the accounting step after the timed ones
    t0 = time.time()
    w = make_workload(name, args.packets, rank, world, args.flows, args.zipf, args.ep_zipf)
    per_ep = per_ep6 = None
    if args.ct_local:
        if name not in ("config3", "config4", "config5"):
            raise SystemExit("--ct-local: configs 3 / 4 / 5")
        per_ep = synth.per_endpoint_ct(w, args.ct_local)
        if name == "config5":                                     # (CT4 and CT6 per endpoint, empty)
            per_ep6 = synth.per_endpoint_ct(w, args.ct_local, "ct6")
    if stateful and per_ep is None:
        size_conntrack(name, w, passes)
        cts = [k for k in ("ct4", "ct6") if k in w.maps and (name != "config3" or k == "ct4")]
        for k in cts:
            if args.ct_room is not None:
                w.maps[k].max_entries = len(np.unique(w.maps[k].keys, axis=0)) + args.ct_room
            if args.ct_max_log2 is not None:
                w.maps[k].max_entries = 1 << args.ct_max_log2
            if args.ct_max is not None:
                w.maps[k].max_entries = args.ct_max
    log(f"[rank {rank}] generated {name}: {w.n} packets in {time.time() - t0:.1f}s")
    ctx, maps = H.product_ctx(w, device=local, ct_per_ep=per_ep, ct6_per_ep=per_ep6)
    log(f"[rank {rank}] tables compiled ({time.time() - t0:.1f}s)")
    metrics_t = torch.zeros(2048, dtype=torch.int64, device=device)
    ctx.metrics_attach(metrics_t)
    n = w.n
    out = {"ret": torch.empty(n, dtype=torch.int32, device=device),
           "identity": torch.empty(n, dtype=torch.int32, device=device)}
    if name == "config1":
        out = {"xdp": torch.empty(n, dtype=torch.uint8, device=device)}
    if stateful:
        out["ct"] = torch.empty(n, dtype=torch.uint8, device=device)

    # the batch of every pass, resident in HBM before anything is timed
    where = None
    if name == "config5":
        parts, where = split_families(w)
        dev_parts = [{k: to_device(v, device) for k, v in p.items()} for p in parts]
        offs = [0, len(parts[0]["length"])]
    else:
        frames, length, mark = H.to_dev(w, device)
    batches = [None] * (passes + 1)
    if stateful:
        base = [p["frames"] for p in dev_parts] if name == "config5" else frames
        for v in range(1, passes + 1):
            batches[v] = step_batch(name, w, v, base, where, device)
        log(f"[rank {rank}] {passes} step batches built on the device ({time.time() - t0:.1f}s)")

    gc_maps = ([maps[k] for k in ("ct4", "ct6") if k in maps] if per_ep is None
               else list(maps["ct4_ep"]) + list(maps.get("ct6_ep", []))) if stateful else []
    gc_deleted = [0]

    def now_of(v):
        return w.now + (v * args.gc_step if args.gc_step else v)

    def step(o, v):
        if args.gc_step:                                           # the agent's ctmap.GC before the batch
            for m in gc_maps:
                gc_deleted[0] += m.ct_gc(now_of(v))
        if name == "config1":
            ctx.xdp_prefilter(frames, length, o)
        elif name == "config2":
            ctx.policy_ingress(0, frames, length, o, mark=mark)
        elif name == "config5":
            for k, (part, off) in enumerate(zip(dev_parts, offs)):
                rows = len(part["length"])
                sub = {kk: t[off:off + rows] for kk, t in o.items()}
                ctx.lxc_egress(batches[v][k], part["length"], sub, now_of(v), src_ep=part["src_ep"],
                               flow_hash=part["flow_hash"])
        else:
            ctx.netdev_ingress(batches[v], length, o, now_of(v), mark=mark)

    v = 1
    for _ in range(args.warmup):
        step(out, v)
        v += 1
    torch.cuda.synchronize()
    log(f"[rank {rank}] warmup done ({time.time() - t0:.1f}s)")

    def full_maps():
        """--ct-local: how many endpoint maps hold max_entries entries (syncs, untimed)"""
        return sum(len(m) >= args.ct_local for m in list(maps["ct4_ep"]) + list(maps.get("ct6_ep", [])))

    def slot_load():
        """live entries / slots of every device CT map (cv_ct_slots; syncs, untimed)"""
        r = {}
        if per_ep is not None:
            return r
        for k in ("ct4", "ct6"):
            if k in maps and stateful:
                e, d, l = maps[k].ct_slots()
                r[k] = round(l / max(e + d + l, 1), 4)
        return r

    load_first = slot_load()
    full_first = full_maps() if per_ep is not None else None
    gc_deleted[0] = 0
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step(out, v)
        ev[i][1].record(stream)
        v += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    step_ms = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(step_ms))
    load_last = slot_load()
    full_last = full_maps() if per_ep is not None else None
    gc_timed = gc_deleted[0]

    # accounting step (untimed, after the timed region, in the same regime): L(p), U(p); the
    # stateful paths count with CV_F_ACCT_SPLIT, which splits out the conntrack lookups and
    # writes (the HBM-resident lines of B(p)) -- pinned equal to the oracle's split in
    # tests/test_gpu_egress.test_acct_split_counts and test_config5_bench_regime
    from cilium_amd import lib
    acct = dict(out)
    acct["nl"] = torch.zeros(n, dtype=torch.uint8, device=device)
    acct["nu"] = torch.zeros(n, dtype=torch.uint8, device=device)
    if stateful:
        ctx.set_flags(lib.F_DEFAULT | lib.F_ACCT_SPLIT)
    step(acct, v)
    torch.cuda.synchronize()
    if stateful:
        ctx.set_flags(lib.F_DEFAULT)
    nl, nu = acct["nl"].cpu().numpy(), acct["nu"].cpu().numpy()
    ct_lines = None
    if stateful:
        U = lib.ACCT_CT_UNIT
        ct_lines = nl.astype(np.int64) // U + nu.astype(np.int64) // U
        nl, nu = nl // U + nl % U, nu // U + nu % U
    created = int((acct["ct"].cpu().numpy() == 0).sum()) if stateful else 0
    hbm_model = hbm_resident_bytes(acct["ct"].cpu().numpy(), acct["ret"].cpu().numpy()) \
        if name in ("config3", "config4") else None
    if name == "config5":
        k4 = offs[1]
        alg_bytes = algorithmic_bytes(name, nl[:k4], nu[:k4], 64) + algorithmic_bytes(name, nl[k4:], nu[k4:], 128)
        hbm_res = k4 * (64 + 9) + (n - k4) * (128 + 9) + 64 * int(ct_lines.sum())
    else:
        alg_bytes = algorithmic_bytes(name, nl, nu)
        hbm_res = n * (64 + 9) + 64 * int(ct_lines.sum()) if stateful else None
    del acct
    log(f"[rank {rank}] accounting step done ({time.time() - t0:.1f}s)")

    local_metrics = metrics_t.cpu().numpy().copy() if args.dump else None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.all_reduce(metrics_t)           # cilium_metrics: the one RCCL reduction
    torch.cuda.synchronize()
    if args.dump:
        from cilium_amd import shard
        os.makedirs(args.dump, exist_ok=True)
        fr = w.frames
        sa = fr[:, 26:30].copy().view("<u4").ravel()
        da = fr[:, 30:34].copy().view("<u4").ravel()
        np.savez(os.path.join(args.dump, f"rank{rank}.npz"), pair_keys=np.unique(shard.pair_key4(sa, da)),
                 metrics_local=local_metrics, metrics_reduced=metrics_t.cpu().numpy(), elapsed=elapsed)

    total_pkts = n * args.steps * world
    value = total_pkts / elapsed / 1e6
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    sha = lib_sha()
    traffic = pmc_traffic(name, sha)

    if rank == 0:
        cpu = None
        ra_peak = None if args.no_cpu else random_access_peak()
        if not args.no_cpu and world == 1:
            log("[rank 0] cpu baseline ...")
            cpu = cpu_baseline(name, w)
            if name in ("config1", "config2"):
                # SURVEY.md §8(d) CPU item (a): the eBPF restatement in the host kernel's
                # own datapath (JIT + kernel LPM/hash maps) via BPF_PROG_TEST_RUN
                log("[rank 0] cpu baseline (kernel eBPF) ...")
                from oracle import kernel_bench
                cpu["kernel_ebpf"] = kernel_bench.run(name, w)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64, SURVEY.md §8(d) seeds), tables + headers resident in HBM",
            "config": {
                "workload": f"{name}: {WORKLOADS[name]}",
                "packets_per_step_per_gpu": n,
                "header_bytes": "64 (v4) / 128 (v6)" if name == "config5" else int(w.frames.shape[1]),
                "parallelism": f"replicated tables, {world} GPU(s), batch per GPU"
                               + (f", conntrack sharded by address pair ({args.flows} flows per GPU of one node-wide set)"
                                  if name in ("config3", "config4") and world > 1 else "")
                               + (", independent CT per rank (N separate nodes: replicas, DESIGN.md §7)"
                                  if name == "config5" and world > 1 else ""),
                "tables": {k: len(m) for k, m in w.maps.items()},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms": round(kern_ms, 4),
                "kernel_ms_min_max": [round(min(step_ms), 4), round(max(step_ms), 4)],
                "algorithmic_bytes_per_launch": alg_bytes,
                "accounting": "L(p), U(p) from an untimed fresh step after the timed ones"
                              + (f" ({created} CT_NEW packets)" if stateful else ""),
                # the same achieved rate against the measured random-access peak (64-B lines,
                # HBM-resident table): > 1 means the tables live in L2 / Infinity Cache
                "random_access": None if ra_peak is None else {
                    "peak": ra_peak, "unit": "GB/s", "frac": round(achieved / ra_peak, 4),
                    "probe": "random 64-B line reads from a 4 GiB HBM table, measured in this run"},
                # the HBM-resident part of the algorithmic bytes (record stream, outputs,
                # conntrack lines) against the same random-line peak; the rest is
                # cache-resident (policy, ipcache, endpoint, prefilter lines)
                "hbm_resident": None if hbm_res is None else {
                    "bytes_per_step": hbm_res, "cache_resident_bytes_per_step": alg_bytes - hbm_res,
                    "achieved": round(hbm_res / (kern_ms * 1e-3) / 1e9, 1), "unit": "GB/s",
                    "frac_random_access": None if ra_peak is None else
                    round(hbm_res / (kern_ms * 1e-3) / 1e9 / ra_peak, 4),
                    "how": "the record stream, the outputs and 64 B per conntrack lookup / write the kernels "
                           "counted (CV_F_ACCT_SPLIT accounting step)",
                    "model_bytes_per_step": hbm_model},
            },
            "cpu_baseline": cpu,
        }
        if stateful and per_ep is not None:
            line["config"]["ct_local"] = {
                "maps": len(per_ep) + len(per_ep6 or []), "max_entries_per_map": args.ct_local,
                "ep_zipf": args.ep_zipf,
                "preloaded_entries": int(sum(len(s) for s in per_ep)),
                "full_maps_first_last_timed_step": [full_first, full_last],
                "how": "ConntrackLocal: every endpoint its own CT4 map (config 5: and CT6 map; "
                       "synth.per_endpoint_ct); launches next to a map's max_entries run admitted (one sorted "
                       "segmented scan over all maps' walks)"}
        elif stateful:
            line["config"]["ct_max_entries"] = {k: int(w.maps[k].max_entries) for k in ("ct4", "ct6") if k in w.maps}
            # live entries / device slots at the first and the last timed step (a table is sized
            # for max_entries at 60 % slot load, so the load tells how far probes walk)
            line["config"]["ct_slot_load"] = {k: [load_first.get(k), load_last.get(k)] for k in load_first}
            if args.zipf:
                from cilium_amd import shard
                fl = w.frames
                pk = shard.pair_key4(fl[:, 26:30].copy().view("<u4").ravel(), fl[:, 30:34].copy().view("<u4").ravel()) \
                    if name in ("config3", "config4") else None
                _, cnt = np.unique(pk, return_counts=True)
                line["config"]["zipf"] = {"a": args.zipf, "largest_pair_packets": int(cnt.max()),
                                          "pairs_over_1000_packets": int((cnt > 1000).sum())}
            if args.gc_step:
                line["config"]["steady_state"] = {
                    "gc_step_s": args.gc_step, "gc_deleted_in_timed_steps": gc_timed,
                    "how": "now advances gc_step seconds per step; ctmap.GC(GCFilterByTime, now) runs before "
                           "every step inside the timed region"}
        os.write(out_fd, (json.dumps(line) + "\n").encode())
    if dist:
        dist.destroy_process_group()
    ctx.close()


def ep_owned(args, rank, world, local, device, dist, out_fd):
    """config 5 as one node across the ranks: a step = the node's rounds over
    one fresh batch -- the scheduler's build (candidates, peers, operations: cv_epnode_open)
    and every round's launches, exchanges and host waits, inside the timed region; the
    batch's records already in HBM and its host copy (what the scheduler reads) built before."""
    import torch
    from cilium_amd import epnode, synth
    from tests import harness as H
    if args.workload != "config5":
        raise SystemExit("--ep-owned: config 5")
    n = args.packets if args.packets != 1 << 24 else 1 << 20
    cap = args.ct_local or 64000
    t0 = time.time()
    w = synth.config5(n, ep_zipf=args.ep_zipf)
    per4 = synth.per_endpoint_ct(w, cap)
    per6 = synth.per_endpoint_ct(w, cap, "ct6")
    ctx, maps = H.product_ctx(w, device=local, ct_per_ep=per4, ct6_per_ep=per6)
    metrics_t = torch.zeros(2048, dtype=torch.int64, device=device)
    ctx.metrics_attach(metrics_t)
    log(f"[rank {rank}] ep-owned config 5: {n} packets, {len(w.endpoints)} endpoints, tables compiled "
        f"({time.time() - t0:.1f}s)")
    xdev = device if args.dist_backend == "nccl" else None         # (gloo: the exchange over host tensors)
    exchange, all_sum = epnode.dist_exchange(world, rank, xdev) if dist else (None, None)
    passes = args.warmup + args.steps + 1
    v6, _ = epnode.families(w.frames)
    batches = []
    for v in range(1, passes + 1):                                 # (fresh client ports per step, built untimed)
        f = H.apply_variant(w.frames, *synth.port_variant(w, v))
        parts = []
        for sel, stride in ((~v6, 64), (v6, 128)):
            idx = np.nonzero(sel)[0]
            parts.append({"frames": torch.from_numpy(np.ascontiguousarray(f[idx, :stride])).to(device),
                          "length": to_device(w.length[idx].astype(np.uint32), device),
                          "src_ep": to_device(w.extra["src_ep"][idx].astype(np.uint16), device),
                          "flow_hash": to_device(w.extra["flow_hash"][idx].astype(np.uint32), device)})
        batches.append((f, parts))
    log(f"[rank {rank}] {passes} step batches built ({time.time() - t0:.1f}s)")

    def step(v):
        f, parts = batches[v - 1]
        node = epnode.EpNode(ctx, rank, world, f, w.length, w.extra["src_ep"], w.extra["flow_hash"], device=device,
                             exchange=exchange, all_sum=all_sum, parts=parts)
        t = time.perf_counter()
        node.run(w.now + v)
        return node, time.perf_counter() - t

    v = 1
    for _ in range(args.warmup):
        step(v)
        v += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    stats, t_run, t_start = [], 0.0, time.perf_counter()
    for _ in range(args.steps):
        node, tr = step(v)
        t_run += tr
        stats.append((node.rounds, node.launches, node.cross, node.sched.stats(), dict(node.times)))
        v += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    # accounting step (untimed): L(p), U(p) of the packets each rank finished
    node, _ = step(v)
    out, idx = node.results()
    rec = np.where(v6[idx], 128, 64)
    alg = int((rec + 9).sum()) + 64 * int(out["nl"].sum() + out["nu"].sum())
    full = sum(len(m) >= cap for m in list(maps["ct4_ep"]) + list(maps["ct6_ep"]))
    if dist:
        t = torch.tensor([elapsed, t_run], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, t_run = float(t[0]), float(t[1])
        a = torch.tensor([alg, sum(s[2] for s in stats), full], dtype=torch.int64, device=device)
        dist.all_reduce(a)
        alg, cross, full = (int(x) for x in a.cpu())
        dist.all_reduce(metrics_t)
    else:
        cross = sum(s[2] for s in stats)
    ms = elapsed * 1e3 / args.steps
    achieved = alg / (ms * 1e-3) / 1e9
    if rank == 0:
        rounds = [s[0] for s in stats]
        line = {
            "metric": METRIC, "value": round(n * args.steps / elapsed / 1e6, 3), "unit": "Mpps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (SplitMix64), tables + headers resident in HBM",
            "config": {
                "workload": "config5 as ONE node across the ranks: endpoint-owned conntrack (ConntrackLocal, every "
                            "endpoint its own CT4 / CT6 map), source programs on the source's rank, deliveries on "
                            "the destination's, records exchanged per round",
                "packets_per_step_node": n, "endpoints": len(w.endpoints), "services": 50000,
                "parallelism": f"{world} rank(s), endpoints e % {world} == rank, one batch per node per step",
                "ct_local": {"maps": len(per4) + len(per6), "max_entries_per_map": cap, "ep_zipf": args.ep_zipf,
                             "full_maps_after": full}},
            "ep_owned": {
                "rounds_per_step": [min(rounds), max(rounds)],
                "launches_per_step_rank0": [min(s[1] for s in stats), max(s[1] for s in stats)],
                "cross_rank_deliveries_per_step": cross // max(args.steps, 1),
                "maps_ordered_whole_first_round_rank0": stats[-1][3]["maps_ordered_whole_at_open"],
                "run_ms_per_step": round(t_run * 1e3 / args.steps, 3),
                "run_ms_split_rank0": {k: round(sum(x[4][k] for x in stats) * 1e3 / args.steps, 3)
                                       for k in stats[0][4]},
                "schedule_build_ms_per_step": round(ms - t_run * 1e3 / args.steps, 3),
                "how": "bench.ep_owned: step = cv_epnode_open (candidates, peers, operations) + EpNode.run "
                       "(per round: split launches, exchange, delivery launches; one host wait)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                         "algorithmic_bytes_per_step": alg,
                         "note": "whole node step (host-driven rounds), not one kernel"},
            "cpu_baseline": None,
        }
        os.write(out_fd, (json.dumps(line) + "\n").encode())
    if dist:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
