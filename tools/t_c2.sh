#!/bin/bash
# config-2 parity tests, then A/B bench of library variants
T=${1:-c2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -v -k "config2 or policy_counters" --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/$T/pytest.log
bash tools/ab_config2.sh $T
