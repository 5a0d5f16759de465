set -e
O=gpurun_out/r04hv; mkdir -p $O
b() { n=$1; shift; echo "[$(date +%T)] $n $*" >&2; timeout -k 10 400 python3 -u bench.py --no-cpu "$@" > $O/$n.json 2> $O/$n.err; tail -c 300 $O/$n.json >&2; }
b b_zipf06 --workload config3 --zipf 0.6
b b_zipf11 --workload config3 --zipf 1.1 --steps 5
b b_fulltable3 --workload config3 --ct-room 0
b b_rightsized_gc --workload config3 --ct-max-log2 26 --gc-step 61
b b_ctmax1M_5 --workload config5 --ct-max 1000000
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/session.sh r04h stats=config1 stats=config2
