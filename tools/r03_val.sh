#!/bin/bash
# Validation session: every -m gpu test, the config-3 bench line, and the PMC passes of
# config 3 (the dominant workload) for the traffic summary; each step under its own limit.
set -u
OUT=gpurun_out/${1:-r03q}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "[step $(date +%T)] $name" >&2; timeout -k 10 $lim "$@"; local rc=$?; echo "[step] $name rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
step bench_config3 300 python3 -u bench.py --workload config3 --no-cpu > $OUT/bench_config3.json 2> $OUT/bench_config3.err
step stats_config3 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_config3 -o run --output-format csv -- python3 bench.py --workload config3 --steps 10 --warmup 2 --no-cpu > $OUT/stats_config3.log 2>&1
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step "pmc$i" 240 rocprofv3 --pmc $CTRS -d $OUT/pmc${i}_config3 -o run --output-format csv -- python3 bench.py --workload config3 --steps 3 --warmup 1 --no-cpu > $OUT/pmc${i}_config3.log 2>&1
done
step pmc_cal 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_cal -o run --output-format csv -- python3 tools/pmc_calibrate.py > $OUT/pmc_cal.log 2>&1
exit 0
