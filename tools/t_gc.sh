#!/bin/bash
T=${1:-gc}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -v -k "ct_gc or ct_map_api" --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/$T/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/st -o run --output-format csv -- python3 -u tools/bench_gc.py > gpurun_out/$T/gc.log 2>&1 || { tail -20 gpurun_out/$T/gc.log; exit 1; }
grep flows gpurun_out/$T/gc.log
grep -E "k_ct_gc|Name" gpurun_out/$T/st/run_kernel_stats.csv | cut -d, -f1-4
