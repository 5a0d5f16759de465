set -u
# final device code: the whole -m gpu suite and smoke
bash tools/session.sh r06fin1 tests smoke
