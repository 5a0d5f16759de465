# parity tests (-k expr, or "-" for none), then a timing A/B of library variants on one workload:
#   bash tools/ab_session.sh <tag> <workload> <pytest -k expr | -> <variant>...
set -u
T=$1; shift; W=$1; shift; K=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
if [ "$K" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "$K" -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/$T/pytest.log | head; tail -30 gpurun_out/$T/pytest.log; exit 1; }
  tail -1 gpurun_out/$T/pytest.log
fi
W=$W bash tools/ab_run.sh $T "$@"
