#!/bin/bash
# all GPU tests, then config-1 and config-3 benches with kernel stats
T=${1:-c13}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/$T/pytest.log
for W in config1 config3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/st_$W -o run --output-format csv -- python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu > gpurun_out/$T/b_$W.log 2>&1 || { tail -20 gpurun_out/$T/b_$W.log; exit 1; }
  grep '"metric"' gpurun_out/$T/b_$W.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$W', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  cut -d, -f1-4 gpurun_out/$T/st_$W/run_kernel_stats.csv | head -5
done
