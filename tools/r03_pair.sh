#!/bin/bash
# GPU session helper: config-5 group statistics + bench + kernel trace, then the config-3
# bench + kernel trace; each step under its own limit, a timeout or crash ends the session.
#   usage: bash tools/r03_pair.sh <tag> [tests]
set -u
OUT=gpurun_out/${1:-r03p}
mkdir -p $OUT
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "[step] $name" >&2
    timeout -k 10 $lim "$@"
    local rc=$?
    echo "[step] $name rc=$rc" >&2
    if [ $rc -ge 124 ]; then echo "[step] stopping after $name" >&2; exit $rc; fi
    return 0
}
if [ "${2:-}" = "tests" ]; then
    step tests 420 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ -k "not bench_regime and not rank_shard_full" > $OUT/gpu.log 2>&1
fi
step groups5 200 env CV_GROUP_STATS=1 python -u bench.py --workload config5 --steps 1 --warmup 0 --no-cpu > $OUT/groups5.json 2> $OUT/groups5.log
step bench5 250 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $OUT/bench5.json 2> $OUT/bench5.log
step bench3 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench3.json 2> $OUT/bench3.log
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
step prof5 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof5 -o c5 -- python3 $ROOTD/bench.py --workload config5 --steps 6 --warmup 1 --no-cpu > $ROOTD/$OUT/prof5.log 2>&1
step prof3 240 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof3 -o c3 -- python3 $ROOTD/bench.py --steps 10 --warmup 2 --no-cpu > $ROOTD/$OUT/prof3.log 2>&1
exit 0
