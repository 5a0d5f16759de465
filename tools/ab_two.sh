# two workloads' timing A/B in one call: bash tools/ab_two.sh <tag> "<variants config5>" "<variants config3>"
set -u
T=$1
export TMPDIR=/tmp
W=config5 bash tools/ab_run.sh ${T}_c5 $2 && W=config3 bash tools/ab_run.sh ${T}_c3 $3
