set -u
bash tools/ep_owned_two_ranks.sh gpurun_out/r06q
