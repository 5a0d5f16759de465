"""The kernel-eBPF CPU baseline (oracle/kernel_bench.py) where bpf(2) is permitted:
this build container (root).  The GPU box runs commands unprivileged
(kernel.unprivileged_bpf_disabled=1), so bench.py reports the error there and this
script's output is committed under profiles/ instead.
Usage: python tools/kernel_ebpf_baseline.py <out.json>"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cilium_amd import synth  # noqa: E402
from oracle import kernel_bench  # noqa: E402

res = {"host": {"cpu_model": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                                   if l.startswith("model name")), "?"),
                "cpus": len(os.sched_getaffinity(0))}}
for name, gen in (("config1", synth.config1), ("config2", synth.config2)):
    w = gen(1 << 18)                      # same tables as the bench (generated before packets)
    res[name] = kernel_bench.run(name, w, min_seconds=10.0)
    print(name, res[name], flush=True)
json.dump(res, open(sys.argv[1], "w"), indent=1)
