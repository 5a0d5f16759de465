#!/bin/bash
# A/B of environment settings: per setting a kernel trace of a short bench run
#   usage: bash tools/r03_ab_env.sh <tag> <workload> "<ENV=V ...>" ["<ENV=V ...>" ...]
set -u
T=$1; W=$2; shift 2
OUT=gpurun_out/$T; mkdir -p $OUT
ROOTD=$PWD
cd /tmp && export TMPDIR=/tmp
k=0
for envs in "$@"; do
  k=$((k+1))
  echo "[ab] $k: $envs" >&2
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOTD/$OUT/v$k -o run -- python3 $ROOTD/bench.py --workload $W --steps 5 --warmup 1 --no-cpu > $ROOTD/$OUT/v$k.log 2>&1
  rc=$?
  echo "[ab] $k rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
