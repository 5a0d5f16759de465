#!/bin/bash
# streaming verdict stores: parity of the stateless kernels, A/B against plain stores,
# then bench + kernel stats + PMC passes for every workload on the new device code
set -u
OUT=gpurun_out/r01y
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "config1 or config2 or empty or ipcache or policy" > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
bash tools/ab_libs.sh r01y/ab_nt "config2 config1" - cilium_amd/_lib/libcilium_hip_nont.so || exit 1
bash tools/ab_libs.sh r01y/ab_nt2 "config2 config1" cilium_amd/_lib/libcilium_hip_nont.so - || exit 1
for w in config2 config1 config3 config5; do
  bash tools/gpu_round.sh $w r01y - || exit 1
done
