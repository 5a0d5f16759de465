#!/bin/bash
# GPU session helper (round 3): tests, benches and a kernel trace, each step under its
# own time limit; a step that times out, crashes or aborts ends the session.
set -u
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
step() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "[step] $name" >&2
    timeout -k 10 $lim "$@"
    local rc=$?
    echo "[step] $name rc=$rc" >&2
    if [ $rc -ge 124 ] || [ $rc -ge 128 ]; then echo "[step] stopping after $name" >&2; exit $rc; fi
    return 0
}
step tests 420 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ -k "not bench_regime and not rank_shard_full" > $OUT/gpu.log 2>&1
step bench 200 python -u bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench.json 2> $OUT/bench.log
step bench_full 240 env CV_ADMIT_STATS=1 python -u bench.py --steps 10 --warmup 2 --no-cpu --ct-room 0 > $OUT/bench_full.json 2> $OUT/bench_full.log
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
step prof 240 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof -o c3 -- python3 $ROOTD/bench.py --steps 10 --warmup 2 --no-cpu > $ROOTD/$OUT/prof.log 2>&1
exit 0
