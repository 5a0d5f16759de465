#!/bin/bash
# incremental map updates: parity under agent churn, then the update+sync cost
set -u
OUT=gpurun_out/${1:-inc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread \
    -k "churn or ipcache or config2 or policy_counters or config3 or ct_gc" > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; tail -20 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
timeout -k 10 300 python3 -u tools/sync_cost.py > "$OUT/sync.json" 2> "$OUT/sync.err" || { echo "sync_cost failed"; tail -5 "$OUT/sync.err"; exit 1; }
cat "$OUT/sync.json"
