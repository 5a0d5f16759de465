set -u
bash tools/session.sh r06m tests=ep_zipf_per_endpoint
