#!/bin/bash
# bench lines with both CPU baselines (oracle + kernel eBPF restatement) for configs 2 and 1
set -u
OUT=gpurun_out/${1:-cpu}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 tools/bpf_probe.py > "$OUT/bpf_probe.log" 2>&1 || true
for w in config2 config1; do
  timeout -k 10 400 python3 -u bench.py --workload $w > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" \
      || { echo "bench $w failed rc=$?"; tail -20 "$OUT/bench_$w.err"; exit 1; }
  cat "$OUT/bench_$w.json"
done
