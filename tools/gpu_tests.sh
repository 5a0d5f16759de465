set -u
mkdir -p gpurun_out/r01c
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r01c/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r01c/pytest.log | head -40
tail -40 gpurun_out/r01c/pytest.log | grep -v "^$" | tail -25
exit $rc
