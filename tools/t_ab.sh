#!/bin/bash
# GPU tests, then the A/B timing of library variants
T=${1:-r01}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/$T/pytest.log
bash tools/ab_egress.sh $T
