#!/bin/bash
# Timing A/B of library builds on one box: bench lines for each (workload, lib).
#   usage: bash tools/ab_libs.sh <tag> "<workloads>" lib1.so lib2.so ...   ("-" = the tree's own build)
set -u
TAG=$1; W=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in $W; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    if [ "$L" = "-" ]; then n=head; unset CV_LIB; else export CV_LIB=$PWD/$L; fi
    timeout -k 10 300 python3 -u bench.py --workload "$w" --no-cpu --steps 10 --warmup 2 > "$OUT/$w.$n.json" 2> "$OUT/$w.$n.err" \
        || { echo "bench $w $n failed rc=$?"; tail -5 "$OUT/$w.$n.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" "$OUT/$w.$n.json" "$w" "$n"
  done
done
