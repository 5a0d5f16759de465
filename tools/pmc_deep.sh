#!/bin/bash
# Instruction / wait / texture-path counters for one workload (one counter group per
# rocprofv3 run; each pass under its own hard time limit).
#   usage: bash tools/pmc_deep.sh <workload> <tag> [packets]
W=${1:-config5}; T=${2:-deep}; P=${3:-4194304}
OUT=gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_ANY" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/p$i -o run --output-format csv \
      -- python3 bench.py --workload $W --packets $P --steps 1 --warmup 1 --no-cpu > $OUT/p$i.log 2>&1 \
      || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT
