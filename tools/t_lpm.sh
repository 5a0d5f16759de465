#!/bin/bash
# LPM layout round: parity tests touching the v4 LPM, then config 1/2/3 A/B of the
# DIR-24-8 build (tree) against the 16-8-8 build (CV_LPM_1688).
set -u
OUT=gpurun_out/${1:-lpm}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread \
    -k "config1 or config2 or ipcache or config3_vs" > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; tail -20 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
bash tools/ab_libs.sh "${1:-lpm}" "config2 config1 config3" - cilium_amd/_lib/libcilium_hip_lpm1688.so
