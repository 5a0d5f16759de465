#!/bin/bash
# round end on the final device code: every GPU test, smoke(), the default bench line,
# then bench + kernel stats + PMC passes per workload (profiles/pmc_<workload>.json)
set -u
bash tools/t_final.sh r01z || exit 1
for w in config2 config1 config3 config5; do
  bash tools/gpu_round.sh $w r01z - || exit 1
done
