set -u
bash tools/session.sh r06s tests=seed_sweep
