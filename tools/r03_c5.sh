#!/bin/bash
# GPU session helper (config 5): group-size statistics of one step, the bench, and a
# kernel trace; each step under its own limit, a timeout or crash ends the session.
set -u
OUT=gpurun_out/${1:-r03c5}
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
step groups 200 env CV_GROUP_STATS=1 python -u bench.py --workload config5 --steps 1 --warmup 0 --no-cpu > $OUT/groups.json 2> $OUT/groups.log
step bench 250 python -u bench.py --workload config5 --steps 10 --warmup 2 --no-cpu > $OUT/bench5.json 2> $OUT/bench5.log
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof -o c5 -- python3 $ROOTD/bench.py --workload config5 --steps 6 --warmup 1 --no-cpu > $ROOTD/$OUT/prof.log 2>&1
exit 0
