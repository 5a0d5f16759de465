set -u
# config 5's conntrack components by size (CV_GROUP_STATS), one short run
mkdir -p gpurun_out/r06l
CV_GROUP_STATS=1 timeout -k 10 300 python3 -u bench.py --workload config5 --steps 1 --warmup 0 --no-cpu > gpurun_out/r06l/bench.json 2> gpurun_out/r06l/group_stats.log
