set -u
# kernel statistics of the ep-owned node (how much of a step the device is busy)
bash tools/session.sh r06r stats=config5,--ep-owned,--steps,5
