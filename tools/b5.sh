mkdir -p gpurun_out/r01r
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r01r/pytest.log 2>&1 || { tail -30 gpurun_out/r01r/pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/r01r/pytest.log
for P in 1048576 4194304; do
timeout -k 10 300 python3 -u bench.py --workload config5 --packets $P --steps 3 --warmup 1 --no-cpu >> gpurun_out/r01r/b5.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01r/st5 -o run --output-format csv -- python3 bench.py --workload config5 --packets 4194304 --steps 3 --warmup 1 --no-cpu >> gpurun_out/r01r/b5.log 2>&1
timeout -k 10 200 python3 -u tools/ablate_egress.py > gpurun_out/r01r/ablate.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/r01r/ablate.json'));print({k:v['ms_median'] for k,v in d.items()})"
timeout -k 10 300 python3 -u bench.py --workload config3 --steps 5 --warmup 2 --no-cpu > gpurun_out/r01r/b3.log 2>&1 && tail -1 gpurun_out/r01r/b3.log
