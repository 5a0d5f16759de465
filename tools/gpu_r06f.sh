set -u
bash tools/session.sh r06f ab=config3,main,r05,main,r05
