#!/bin/bash
# Checkpoint session: A = every -m gpu test, smoke, the bench line and kernel statistics of
# configs 3/5/1/2; B = PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) of configs 3/5 and
# the random-line calibration.  Each GPU step has its own limit; a failure ends the session.
#   usage: bash tools/r03_ckpt.sh <tag> A|B
set -u
TAG=$1; PART=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
ROOTD=$PWD
export TMPDIR=/tmp
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "[step $(date +%T)] $name" >&2
    timeout -k 10 $lim "$@"
    local rc=$?
    echo "[step] $name rc=$rc" >&2
    if [ $rc -ne 0 ]; then echo "[step] stopping after $name" >&2; exit $rc; fi
}
if [ "$PART" = "A" ]; then
    step tests 700 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
    step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
    for W in config3 config5 config1 config2; do
        step bench_$W 300 python3 -u bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err
        step stats_$W 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_$W -o run --output-format csv \
            -- python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu > $OUT/stats_$W.log 2>&1
    done
else
    for W in config3 config5; do
        i=0
        for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
            i=$((i+1))
            step "pmc$i $W" 240 rocprofv3 --pmc $CTRS -d $OUT/pmc${i}_$W -o run --output-format csv \
                -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu > $OUT/pmc${i}_$W.log 2>&1
        done
    done
    step pmc_cal 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_cal -o run --output-format csv \
        -- python3 tools/pmc_calibrate.py > $OUT/pmc_cal.log 2>&1
fi
exit 0
