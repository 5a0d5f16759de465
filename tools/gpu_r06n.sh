set -u
# deep counters (SQ / TA / TCP) of the final device code's config 3 and config 5 kernels
bash tools/session.sh r06n deep=config3 deep=config5
