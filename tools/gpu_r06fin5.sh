set -u
# the final tree with the seed sweep: whole -m gpu suite + smoke
bash tools/session.sh r06fin5 tests smoke
