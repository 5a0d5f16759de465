set -u
# the final tree (host-side scheduler changes and the new tests on the frozen device code): whole -m gpu suite + smoke
bash tools/session.sh r06fin4 tests smoke
