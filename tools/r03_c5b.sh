#!/bin/bash
# GPU session (config 5): egress parity tests, group statistics, bench, kernel trace
set -u
OUT=gpurun_out/${1:-r03c5b}
K=${2:-egress or config5}
mkdir -p $OUT
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "[step] $name" >&2
    timeout -k 10 $lim "$@"
    local rc=$?
    echo "[step] $name rc=$rc" >&2
    if [ $rc -ne 0 ]; then echo "[step] stopping after $name" >&2; exit $rc; fi
    return 0
}
if [ "$K" != "-" ]; then
step tests 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ -k "$K" > $OUT/gpu.log 2>&1
fi
step groups5 200 env CV_GROUP_STATS=1 python -u bench.py --workload config5 --steps 1 --warmup 0 --no-cpu > $OUT/groups5.json 2> $OUT/groups5.log
step bench5 250 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $OUT/bench5.json 2> $OUT/bench5.log
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
step prof5 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof5 -o c5 -- python3 $ROOTD/bench.py --workload config5 --steps 6 --warmup 1 --no-cpu > $ROOTD/$OUT/prof5.log 2>&1
exit 0
