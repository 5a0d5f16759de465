set -u
mkdir -p gpurun_out/pmc5
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS -d gpurun_out/pmc5/p$i -o run --output-format csv -- python3 tools/egress_once.py > gpurun_out/pmc5/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc5/p$i.log; exit 1; }
done
echo done
