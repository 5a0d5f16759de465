set -u
bash tools/session.sh r06e tests=ep_node,or,room_bound,or,ep_owned bench=config3 bench=config5,--ep-owned,--steps,3,--warmup,1,--no-cpu bench=config3,--ct-local,64000,--ep-zipf,1.0,--steps,5,--warmup,2,--no-cpu bench=config5,--ct-local,64000,--ep-zipf,0.6,--steps,5,--warmup,2,--no-cpu
