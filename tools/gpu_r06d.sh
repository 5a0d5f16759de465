set -u
bash tools/session.sh r06d tests=room_bound,or,acct_split,or,ep_node,or,config5_bench_regime,or,config5_per_endpoint bench=config3,--steps,10,--warmup,2,--no-cpu bench=config5,--steps,10,--warmup,2,--no-cpu bench=config3,--ct-local,64000,--ep-zipf,1.0,--steps,5,--warmup,2,--no-cpu bench=config5,--ep-owned,--steps,3,--warmup,1,--no-cpu || exit $?
mkdir -p gpurun_out/r06d
CV_ADMIT_STATS=1 timeout -k 10 300 python3 bench.py --workload config5 --ct-local 64000 --steps 3 --warmup 1 --no-cpu > gpurun_out/r06d/c5local.json 2> gpurun_out/r06d/c5local.err
