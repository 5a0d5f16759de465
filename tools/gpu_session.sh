#!/bin/bash
# One GPU-box session: the -m gpu tests, the bench line, and the rocprofv3 kernel
# summary of one workload.  Every GPU step has its own time limit and the chain stops
# at the first failure.
#   usage: bash tools/gpu_session.sh <tag> <workload> [pytest -k expr | all | -] [pmc]
# With "pmc" the counter passes follow (one counter group per rocprofv3 run, each under
# a hard limit): FETCH_SIZE, WRITE_SIZE, TCC hit/miss, and SQ instruction/wait counts;
# tools/pmc_summary.py <tag> <workload> turns them into profiles/.
set -u
TAG=${1:-r02}
W=${2:-config3}
K=${3:-all}
PMC=${4:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ "$K" != "-" ]; then
  step pytest
  if [ "$K" = "all" ]; then KARG=(); else KARG=(-k "$K"); fi
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${KARG[@]}" \
      > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; tail -30 "$OUT/pytest.log"; exit 1; }
  grep -cE "PASSED" "$OUT/pytest.log"
fi
step bench
timeout -k 10 600 python3 -u bench.py --workload "$W" > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench_$W.err"; exit 1; }
cat "$OUT/bench_$W.json"
step rocprof-stats
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$W" -o run --output-format csv \
    -- python3 bench.py --workload "$W" --steps 10 --warmup 2 --no-cpu > "$OUT/stats_$W.log" 2>&1 \
    || { echo "rocprof stats failed rc=$?"; tail -20 "$OUT/stats_$W.log"; exit 1; }
find "$OUT/stats_$W" -name "*kernel_stats.csv" -exec cp {} "$OUT/${W}_kernel_stats.csv" \;
head -12 "$OUT/${W}_kernel_stats.csv"
if [ "$PMC" = "pmc" ]; then
  i=0
  for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
              "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    step "pmc $CTRS"
    timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$OUT/pmc${i}_$W" -o run --output-format csv \
        -- python3 bench.py --workload "$W" --steps 3 --warmup 1 --no-cpu > "$OUT/pmc${i}_$W.log" 2>&1 \
        || { echo "pmc pass $i failed rc=$?"; tail -20 "$OUT/pmc${i}_$W.log"; exit 1; }
  done
  step "pmc calibration (random 64-B lines)"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_cal" -o run --output-format csv \
      -- python3 tools/pmc_calibrate.py > "$OUT/pmc_cal.log" 2>&1 \
      || { echo "pmc calibration failed rc=$?"; tail -20 "$OUT/pmc_cal.log"; exit 1; }
fi
step done
