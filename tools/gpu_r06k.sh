set -u
# the scheduler's host changes: its GPU tests and the ep-owned bench line (device code unchanged)
bash tools/session.sh r06k tests=ep_node,or,ep_owned,or,at_capacity,or,fresh_context bench=config5,--ep-owned
