set -u
# the scheduler's parallel map order and level split: its GPU tests and the ep-owned line
bash tools/session.sh r06o tests=ep_node,or,ep_owned,or,at_capacity,or,fresh_context bench=config5,--ep-owned
