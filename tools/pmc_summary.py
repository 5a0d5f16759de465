#!/usr/bin/env python3
"""Summarise one `tools/gpu_session.sh <tag> <workload> <k> pmc` run (gpurun_out/<tag>/) into committed profiles:

  profiles/<tag>/<workload>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>/bench_<workload>.json         the bench line of that run
  profiles/pmc_<workload>.json                 per-launch PMC counters of the dominant
                                               kernel + lib_sha (read by bench.py)

HBM traffic per launch follows MI355X_MICROARCH.md § HBM: FETCH_SIZE (KiB) doubled
(gfx950 tallies 128-B requests at 64 B) plus WRITE_SIZE (KiB).  Both derive from the
L2's memory-side requests, so Infinity-Cache hits are included.

  usage: python tools/pmc_summary.py <tag> <workload>
"""
import csv
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = {"config1": "k_xdp_prefilter", "config2": "k_policy_ingress", "config3": "k_ct_stage<false>",
            "config5": "k_egress_ct<false, false>"}


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
    kname = DOMINANT[w]
    ctr = {}
    for i in (1, 2, 3):
        p = os.path.join(src, f"pmc{i}_{w}", "run_counter_collection.csv")
        for name, cs in per_kernel(p).items():
            if f"::{kname}(" in name:
                for c, v in cs.items():
                    # config 5's v6 launch also runs the v4 stage kernels on empty
                    # queues: such near-empty dispatches are not launches of the path
                    v = [x for x in v if x >= 0.01 * max(v)] or v
                    ctr[c] = (sum(v) / len(v), len(v))
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
        "dispatches_per_pass": ctr["FETCH_SIZE"][1],
        "rocprof_avg_kernel_ns": avg_ns,
        "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
        "TCC_HIT_sum": hit, "TCC_MISS_sum": miss, "l2_hit_rate": round(hit / (hit + miss), 4),
        "hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
        "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section); memory-side bytes incl. Infinity-Cache hits",
    }
    json.dump(out, open(os.path.join(ROOT, "profiles", f"pmc_{w}.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
