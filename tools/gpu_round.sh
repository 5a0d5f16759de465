#!/bin/bash
# One GPU-box session: parity tests, the bench line, the rocprofv3 kernel summary and
# the PMC passes (one counter group per run) for one workload.  Every GPU step has its
# own time limit and the chain stops at the first failure.
#   usage: bash tools/gpu_round.sh <workload> <tag> [pytest -k expr|-]
set -u
W=${1:-config2}
TAG=${2:-r01}
K=${3:--}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }

if [ "$K" != "-" ]; then
  step pytest
  if [ "$K" = "all" ]; then KARG=(); else KARG=(-k "$K"); fi
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread "${KARG[@]}" \
      > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
  grep -cE "PASSED" "$OUT/pytest.log"
fi

step bench
timeout -k 10 300 python3 -u bench.py --workload "$W" > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_$W.err"; exit 1; }
cat "$OUT/bench_$W.json"

step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$W" -o run --output-format csv \
    -- python3 bench.py --workload "$W" --steps 10 --warmup 2 --no-cpu > "$OUT/stats_$W.log" 2>&1 \
    || { echo "rocprof stats failed rc=$?"; tail -20 "$OUT/stats_$W.log"; exit 1; }

i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step "pmc $CTRS"
  timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$OUT/pmc${i}_$W" -o run --output-format csv \
      -- python3 bench.py --workload "$W" --steps 3 --warmup 1 --no-cpu > "$OUT/pmc${i}_$W.log" 2>&1 \
      || { echo "pmc pass $i failed rc=$?"; tail -20 "$OUT/pmc${i}_$W.log"; exit 1; }
done
step done
