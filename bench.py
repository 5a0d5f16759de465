#!/usr/bin/env python3
"""Benchmark of the MI355X batch verdict engine (BASELINE.json metric).

A step = one pass of the verdict path over one batch of synthetic packets already
resident in HBM.  Default workload = BASELINE.json configs[1] (config 2): ipcache
LPM (102,401 CIDRs -> identities) + policymap (10k identities x 8 L4 ports + L3 +
wildcards, 81,055 entries) ingress verdicts on 2^24 64-B IPv4 headers per step, one
MI355X per rank.  --workload config1 / config3 measure the other paths.

Multi-GPU (torchrun): tables are replicated, every rank verdicts its own batch
(weak scaling, no data-path collective); cilium_metrics is summed across ranks
with one RCCL all_reduce after the timed region.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "Mpps verdicts at 1/2/4/8 GPUs (64B hdrs); achieved HBM GB/s vs peak"

WORKLOADS = {
    "config2": "ipcache LPM (100k CIDRs->identities) + policymap (10k identities x L4 ports) ingress verdicts",
    "config1": "bpf_xdp.c CIDR deny-list prefilter, 1k IPv4 prefixes + cilium_lxc",
    "config3": "full bpf_lxc ingress path: prefilter + ipcache + lxc + policy + ct_lookup4/ct_create4, 16M-flow CT",
    "config4": "config 3 per GPU with conntrack sharded by address pair (16M flows per GPU, 128M on 8), "
               "RCCL all_reduce of cilium_metrics",
    "config5": "dual-stack from-container egress: lb4/lb6 (50k services) + CT4/CT6 + egress policy + local delivery "
               "(v4 64-B and v6 128-B records, 1:1)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def lib_sha():
    """the device code the PMC summaries were taken with (cilium_amd/build.py kernel_sha);
    an A/B library (CV_LIB) is keyed by its own file hash"""
    from cilium_amd import build, lib
    if os.environ.get("CV_LIB"):
        with open(lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    return build.kernel_sha()


def make_workload(name, n, rank):
    from cilium_amd import synth
    if name == "config2":
        return synth.config2(n)
    if name == "config1":
        return synth.config1(n)
    if name == "config3":
        return synth.config3(n, n_flows=1 << 24)
    if name == "config4":
        # the rank's shard: flows whose address pair hashes to it (pre-steered by the producer)
        return synth.config3(n, n_flows=1 << 24, seed=0xC1A00004 + 7919 * rank)
    if name == "config5":
        return synth.config5(n)
    raise SystemExit(f"unknown workload {name}")


def split_families(w):
    """config 5: the v4 packets as 64-B records and the v6 packets as 128-B records
    (two launches per step; v4 and v6 state are disjoint, so order between them is free)."""
    import numpy as np
    v6 = w.extra["v6"]
    parts = []
    for sel, stride in ((~v6, 64), (v6, 128)):
        idx = np.nonzero(sel)[0]
        parts.append({"frames": np.ascontiguousarray(w.frames[idx, :stride]), "length": w.length[idx],
                      "src_ep": w.extra["src_ep"][idx], "flow_hash": w.extra["flow_hash"][idx]})
    return parts


def algorithmic_bytes(name, nl, nu, record=64):
    """B(p) = R + V + 64*L(p) + 64*U(p), summed over the batch."""
    R = record
    V = {"config1": 4, "config2": 8, "config3": 9, "config4": 9, "config5": 9}[name]
    n = len(nl)
    return n * (R + V) + 64 * (int(nl.astype(np.int64).sum()) + int(nu.astype(np.int64).sum()))


def cpu_baseline(name, w, min_seconds=10.0):
    """The oracle (plain-C restatement) timed on the host cores on a bounded sample
    of the same workload (>= min_seconds of CPU work): OpenMP over the cores for the
    stateless paths (configs 1, 2), one thread in packet order for the stateful ones
    (conntrack: configs 3-5), re-running the sample until the time is reached."""
    from tests import harness as H
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    sample = min(w.n, 1 << 21)
    dp, _ = H.oracle_dp(w)
    frames, length, mark = w.frames[:sample], w.length[:sample], w.mark[:sample]
    if name == "config1":
        run = lambda: dp.xdp_prefilter(frames, length)
    elif name == "config2":
        run = lambda: dp.policy_ingress(0, frames, length, mark)
    elif name == "config5":
        sample = min(sample, 1 << 18)
        src, fh = w.extra["src_ep"][:sample], w.extra["flow_hash"][:sample]
        frames, length = frames[:sample], length[:sample]
        run = lambda: dp.lxc_egress(frames, length, src, fh, now=w.now)
    else:
        sample = min(sample, 1 << 18)
        frames, length, mark = frames[:sample], length[:sample], mark[:sample]
        run = lambda: dp.netdev_ingress(frames, length, mark, now=w.now)
    # stateful paths re-run the same sample: later passes see the flows the first created
    done, t0 = 0, time.perf_counter()
    while True:
        run()
        done += sample
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    seq = name in ("config3", "config4", "config5")
    return {"value": round(done / el / 1e6, 3), "unit": "Mpps", "cores": 1 if seq else threads,
            "kind": "port",
            "sample": f"oracle/cv_oracle.c over {done} packets of the same synthetic {name} batch "
                      f"({el:.1f} s, {'1 thread, sequential (stateful path)' if seq else 'OpenMP ' + str(threads) + ' threads'})"}


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
    """HBM bytes per launch from the committed rocprofv3 --pmc summary of this exact
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
    return d.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="config2", choices=sorted(WORKLOADS))
    ap.add_argument("--packets", type=int, default=1 << 24)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg and the random-access probe (profiling runs)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = f"cuda:{local}"
    torch.cuda.set_device(local)

    from cilium_amd import build as cvbuild
    cvbuild.build()
    from tests import harness as H

    name = args.workload
    t0 = time.time()
    w = make_workload(name, args.packets, rank)
    log(f"[rank {rank}] generated {name}: {w.n} packets in {time.time() - t0:.1f}s")
    ctx, maps = H.product_ctx(w, device=local)
    log(f"[rank {rank}] tables compiled ({time.time() - t0:.1f}s)")
    metrics_t = torch.zeros(2048, dtype=torch.int64, device=device)
    ctx.metrics_attach(metrics_t)
    n = w.n
    out = {"ret": torch.empty(n, dtype=torch.int32, device=device),
           "identity": torch.empty(n, dtype=torch.int32, device=device)}
    if name == "config1":
        out = {"xdp": torch.empty(n, dtype=torch.uint8, device=device)}
    if name in ("config3", "config4", "config5"):
        out["ct"] = torch.empty(n, dtype=torch.uint8, device=device)
    if name == "config5":
        parts = []
        for part in split_families(w):
            t = {}
            for k, v in part.items():
                if v.dtype == np.uint16 or (k == "flow_hash" and v.dtype == np.uint32):
                    v = v.view(np.int16 if v.dtype == np.uint16 else np.int32)
                t[k] = torch.from_numpy(np.ascontiguousarray(v)).to(device)
            t["rows"] = len(part["length"])
            parts.append(t)
        offs = [0, parts[0]["rows"]]
    else:
        frames, length, mark = H.to_dev(w, device)

    def step(o):
        if name == "config1":
            ctx.xdp_prefilter(frames, length, o)
        elif name == "config2":
            ctx.policy_ingress(0, frames, length, o, mark=mark)
        elif name == "config5":
            for part, off in zip(parts, offs):
                sub = {k: v[off:off + part["rows"]] for k, v in o.items()}
                ctx.lxc_egress(part["frames"], part["length"], sub, w.now, src_ep=part["src_ep"],
                               flow_hash=part["flow_hash"])
        else:
            ctx.netdev_ingress(frames, length, o, w.now, mark=mark)

    # accounting pass (untimed): L(p), U(p) of the same batch for the algorithmic bytes
    acct = dict(out)
    acct["nl"] = torch.zeros(n, dtype=torch.uint8, device=device)
    acct["nu"] = torch.zeros(n, dtype=torch.uint8, device=device)
    step(acct)
    torch.cuda.synchronize()
    nl, nu = acct["nl"].cpu().numpy(), acct["nu"].cpu().numpy()
    log(f"[rank {rank}] accounting pass done ({time.time() - t0:.1f}s)")
    if name == "config5":
        k4 = offs[1]
        alg_bytes = algorithmic_bytes(name, nl[:k4], nu[:k4], 64) + algorithmic_bytes(name, nl[k4:], nu[k4:], 128)
    else:
        alg_bytes = algorithmic_bytes(name, nl, nu)
    del acct

    for _ in range(args.warmup):
        step(out)
    torch.cuda.synchronize()
    log(f"[rank {rank}] warmup done ({time.time() - t0:.1f}s)")

    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step(out)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.all_reduce(metrics_t)           # cilium_metrics: the one RCCL reduction
    torch.cuda.synchronize()

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
                "parallelism": f"replicated tables, {world} GPU(s), batch per GPU",
                "tables": {k: len(v) for k, v in w.maps.items()},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": alg_bytes,
                # the same achieved rate against the measured random-access peak (64-B lines,
                # HBM-resident table): > 1 means the tables live in L2 / Infinity Cache
                "random_access": None if ra_peak is None else {
                    "peak": ra_peak, "unit": "GB/s", "frac": round(achieved / ra_peak, 4),
                    "probe": "random 64-B line reads from a 4 GiB HBM table, measured in this run"},
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
