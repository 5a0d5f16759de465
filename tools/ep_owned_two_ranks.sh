#!/bin/bash
# bench.py --ep-owned at N = 2 on one GPU (two ranks on GPU 0, gloo): config 5's own node
# (4 096 endpoints, 8 192 per-endpoint maps, 2^20 packets per step) split over two ranks --
# the rounds, the per-round exchange of delivery records and the cross-rank deliveries at
# full size (throughput is not a scaling figure: both ranks share one GPU).
#   usage: bash tools/ep_owned_two_ranks.sh <out dir>
set -u
OUT=$1
mkdir -p "$OUT"
PORT=$((20000 + RANDOM % 20000))
pids=()
for r in 0 1; do
  WORLD_SIZE=2 RANK=$r LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
    timeout -k 10 900 python3 -u bench.py --gpus 2 --workload config5 --ep-owned --steps 3 --warmup 1 \
    --dist-backend gloo > "$OUT/rank$r.json" 2> "$OUT/rank$r.err" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
exit $rc
