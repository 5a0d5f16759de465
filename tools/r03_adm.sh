#!/bin/bash
# GPU session helper: the stream/ipcache tests, then a kernel trace of the full-table
# (admission) bench; each step under its own limit, a timeout or crash ends the session.
set -u
OUT=gpurun_out/${1:-r03adm}
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
step tests 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/ -k "${2:-ipcache or stream_without}" > $OUT/gpu.log 2>&1
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/prof -o full -- python3 $ROOTD/bench.py --steps 4 --warmup 1 --no-cpu --ct-room 0 > $ROOTD/$OUT/prof.log 2>&1
exit 0
