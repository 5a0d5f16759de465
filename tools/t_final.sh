#!/bin/bash
# round-end rehearsal: every GPU test, smoke(), the default bench line
set -u
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; tail -20 "$OUT/pytest.log"; exit 1; }
grep -cE "PASSED" "$OUT/pytest.log"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
