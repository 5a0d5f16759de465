#!/bin/bash
# policy memo round: conntrack-path parity tests on the tree's build, then config 5/3
# A/B against the build without the memo (CV_NO_POLMEMO)
set -u
OUT=gpurun_out/${1:-memo}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_egress.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread \
    -k "config5 or config3 or empty" > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; tail -20 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
bash tools/ab_libs.sh "${1:-memo}" "config5 config3" - cilium_amd/_lib/libcilium_hip_nomemo.so
