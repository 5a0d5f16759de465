#!/bin/bash
# Build the HIP library of an older commit (timing A/B only; run with CV_LIB=<out>):
#   bash tools/build_old_lib.sh <commit> <out.so>
set -e
C=$1; OUT=$2
T=$(mktemp -d)
git -C "$(dirname "$0")/.." archive "$C" cilium_amd/csrc include | tar -x -C "$T"
objs=()
for f in "$T"/cilium_amd/csrc/*.hip "$T"/cilium_amd/csrc/*.cpp; do
  o="$T/$(basename "$f").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -c -x hip "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$OUT"
rm -rf "$T"
