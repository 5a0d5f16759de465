set -u
bash tools/session.sh r06i tests=ep_node,or,room_bound,or,acct_split,or,overcounted,or,config5_bench_regime,or,fresh_context,or,at_capacity \
 && CV_ADMIT_STATS=1 bash tools/session.sh r06i bench=config5,--ct-local,64000,--steps,5,--warmup,1,--no-cpu \
 && CV_ADMIT_STATS=1 bash tools/session.sh r06i bench=config5,--ct-local,64000,--ep-zipf,0.6,--steps,5,--warmup,1,--no-cpu
