mkdir -p gpurun_out/dbg
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_egress.py -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/dbg/t.log 2>&1
grep -E "MISMATCH|PASSED|FAILED" gpurun_out/dbg/t.log | cut -c1-600 | head -30
