#!/usr/bin/env python3
"""Summarise one `tools/session.sh <tag> pmc=<workload> cal` run (gpurun_out/<tag>/) into committed profiles:

  profiles/<tag>/<workload>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>/bench_<workload>.json         the bench line of that run
  profiles/pmc_<workload>.json                 per-launch PMC counters of the dominant
                                               kernel + lib_sha (read by bench.py)

HBM traffic per launch follows MI355X_MICROARCH.md § HBM: FETCH_SIZE (KiB) doubled
(gfx950 tallies 128-B requests at 64 B) plus WRITE_SIZE (KiB).  Both derive from the
L2's memory-side requests, so Infinity-Cache hits are included.

  usage: python tools/pmc_summary.py <tag> <workload> [kernel]   (default: the largest total time)
"""
import csv
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETUP = ("k_ct_load", "k_ct_scan", "k_ct_op", "k_ct_gc", "k_ct_tags")   # table loads, map API, slot-load probe


def dominant(stats_csv):
    """the kernel with the largest total time in the kernel statistics (the step's
    dominant kernel), as its name between `cv::` and the argument list"""
    best, name = -1.0, None
    for r in csv.DictReader(open(stats_csv)):
        n = r["Name"]
        if not n.startswith(("cv::", "void cv::")) or any(f"::{x}(" in n for x in SETUP):
            continue
        if float(r["TotalDurationNs"]) > best:
            best, name = float(r["TotalDurationNs"]), n
    short = name.split("cv::", 1)[1]
    return short[:short.index("(")] if "(" in short else short
# a kernel launched exactly once per step (counts the steps of a pass)
STEP_KERNEL = {"config1": "k_xdp_prefilter", "config2": "k_policy_ingress", "config3": "k_netdev_front<false>",
               "config5": "k_egress_front<32, false>"}


def per_kernel(path):
    d = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    tag, w = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, f"stats_{w}", "run_kernel_stats.csv"), os.path.join(dst, f"{w}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, f"bench_{w}.json"), os.path.join(dst, f"bench_{w}.json"))
    kname = sys.argv[3] if len(sys.argv) > 3 else dominant(os.path.join(src, f"stats_{w}", "run_kernel_stats.csv"))
    setup = SETUP
    ctr, step = {}, defaultdict(float)
    nsteps = 0
    for i in (1, 2, 3):
        p = os.path.join(src, f"pmc{i}_{w}", "run_counter_collection.csv")
        for name, cs in per_kernel(p).items():
            if i == 1 and f"::{STEP_KERNEL[w]}(" in name:
                nsteps = len(next(iter(cs.values())))
            if not name.startswith(("cv::", "void cv::")) or any(f"::{x}(" in name for x in setup):
                continue
            for c, v in cs.items():
                step[c] += sum(v)                                 # every dispatch of the step's kernels
            if f"::{kname}(" in name:
                for c, v in cs.items():
                    # config 5's v6 launch also runs the v4 stage kernels on empty
                    # queues: such near-empty dispatches are not launches of the path
                    v = [x for x in v if x >= 0.01 * max(v)] or v
                    ctr[c] = (sum(v) / len(v), len(v))
    steps = nsteps or ctr["FETCH_SIZE"][1]
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, f"stats_{w}", "run_kernel_stats.csv")))}
    avg_ns = next(float(r["AverageNs"]) for n, r in stats.items() if f"::{kname}(" in n)
    tp = os.path.join(src, f"stats_{w}", "run_kernel_trace.csv")
    if os.path.exists(tp):                                        # same filter on the durations
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(tp))
             if f"::{kname}(" in r["Kernel_Name"]]
        d = [x for x in d if x >= 0.01 * max(d)] or d
        avg_ns = sum(d) / len(d)
    fetch, write = ctr["FETCH_SIZE"][0], ctr["WRITE_SIZE"][0]
    hit, miss = ctr["TCC_HIT_sum"][0], ctr["TCC_MISS_sum"][0]
    sys.path.insert(0, ROOT)
    from cilium_amd import build
    sha = build.kernel_sha()
    out = {
        "workload": w, "kernel": kname, "tag": tag, "kernel_sha": sha,
        "dispatches_per_pass": steps,
        "rocprof_avg_kernel_ns": avg_ns,
        "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
        "TCC_HIT_sum": hit, "TCC_MISS_sum": miss, "l2_hit_rate": round(hit / (hit + miss), 4),
        "hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
        "step_FETCH_SIZE_KiB": step["FETCH_SIZE"] / steps, "step_WRITE_SIZE_KiB": step["WRITE_SIZE"] / steps,
        "hbm_bytes_per_step": int((2 * step["FETCH_SIZE"] + step["WRITE_SIZE"]) * 1024 / steps),
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section); memory-side bytes incl. "
                      "Infinity-Cache hits; per launch of the dominant kernel, and per step = every cv:: kernel "
                      "of the step (table loads excluded) / steps in the pass",
    }
    cal = os.path.join(src, "pmc_cal", "run_counter_collection.csv")
    if os.path.exists(cal):                                       # known bytes / counter, random 64-B lines
        fs = [v for cs in per_kernel(cal).values() for v in cs.get("FETCH_SIZE", [])]
        if fs:
            out["fetch_calibration_random64"] = round((1 << 26) * 64 / (max(fs) * 1024), 3)
            out["hbm_bytes_per_step_calibrated"] = int((out["fetch_calibration_random64"] * step["FETCH_SIZE"]
                                                        + step["WRITE_SIZE"]) * 1024 / steps)
    json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{w}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
