#!/bin/bash
# config-2 timing-only ablations (CV_ABLATE bits, cilium_amd/csrc/cv_dp.hpp)
T=${1:-abl2}
mkdir -p gpurun_out/$T
for A in 0 1 2 4 8 6; do
  CV_ABLATE=$A timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/$T/a$A.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/$T/a$A.log').read().strip().splitlines()[-1]);print('ablate $A', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
