#!/bin/bash
# egress parity tests, then the egress ablation timing
T=${1:-eg}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_egress.py tests/test_multi_rank.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/$T/pytest.log
timeout -k 10 200 python3 -u tools/ablate_egress.py > gpurun_out/$T/a.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/$T/a.json'));print({k:v['ms_median'] for k,v in d.items()})"
