#!/bin/bash
# 64-B CT4 bucket variant: parity of the conntrack tests with the variant library, then
# config 3 / 5 A/B against the tree's build
set -u
OUT=gpurun_out/${1:-ct64}
mkdir -p "$OUT"
export TMPDIR=/tmp
CV_LIB=$PWD/cilium_amd/_lib/libcilium_hip_ct64.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_egress.py -m gpu -v --timeout 200 --timeout-method thread \
    -k "config3 or ct_gc or ct_map or config5_dual or hot_flows" > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; tail -20 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
bash tools/ab_libs.sh "${1:-ct64}" "config3 config5" - cilium_amd/_lib/libcilium_hip_ct64.so
