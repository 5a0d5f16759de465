#!/bin/bash
# Bench lines (+ rocprofv3 kernel stats) for the given workloads, one GPU step per
# command with its own time limit; stops at the first failure.
#   usage: bash tools/gpu_bench.sh <tag> <workload>...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for W in "$@"; do
  echo "[$(date +%T)] bench $W"
  timeout -k 10 400 python3 -u bench.py --workload "$W" ${BENCH_ARGS:-} > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
      || { echo "bench $W failed rc=$?"; tail -20 "$OUT/bench_$W.err"; exit 1; }
  cat "$OUT/bench_$W.json"
  echo "[$(date +%T)] rocprof $W"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$W" -o run --output-format csv \
      -- python3 bench.py --workload "$W" --steps 5 --warmup 1 --no-cpu > "$OUT/stats_$W.log" 2>&1 \
      || { echo "rocprof $W failed rc=$?"; tail -20 "$OUT/stats_$W.log"; exit 1; }
  head -12 "$OUT/stats_$W/run_kernel_stats.csv" | cut -c1-200
done
echo "[$(date +%T)] done"
