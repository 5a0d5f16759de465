#!/bin/bash
# A/B timing of library variants (tools/build_variants.sh): config-5 egress ablations
# and the config-3 bench, one library at a time.
T=${1:-ab}
mkdir -p gpurun_out/$T
for L in ${LIBS:-libcilium_hip libcilium_hip_eg1 libcilium_hip_eg2 libcilium_hip_eg3}; do
  CV_LIB=$PWD/cilium_amd/_lib/$L.so timeout -k 10 200 python3 -u tools/ablate_egress.py > gpurun_out/$T/$L.json 2>/dev/null || exit 1
  echo $L; python3 -c "import json;d=json.load(open('gpurun_out/$T/$L.json'));print({k:v['ms_median'] for k,v in d.items()})"
  [ -n "$B3" ] && { CV_LIB=$PWD/cilium_amd/_lib/$L.so timeout -k 10 200 python3 -u bench.py --workload config3 --steps 5 --warmup 2 --no-cpu > gpurun_out/$T/$L.b3.log 2>&1 || exit 1; }
  [ -n "$B3" ] && python3 -c "import json;d=json.loads(open('gpurun_out/$T/$L.b3.log').read().strip().splitlines()[-1]);print('config3', d['value'], d['ms_per_step'])"
done
true
