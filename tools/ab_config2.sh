#!/bin/bash
# A/B timing of library variants on the default (config 2) bench
T=${1:-ab2}
mkdir -p gpurun_out/$T
for L in ${LIBS:-libcilium_hip}; do
  CV_LIB=$PWD/cilium_amd/_lib/$L.so timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/$T/$L.b2.log 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/$T/$L.b2.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
