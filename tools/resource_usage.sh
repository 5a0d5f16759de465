#!/bin/bash
# Register / LDS / scratch / occupancy per kernel of the HIP sources in a tree:
#   bash tools/resource_usage.sh [repo root (default: this tree)]
ROOT=${1:-$(cd "$(dirname "$0")/.." && pwd)}
T=$(mktemp -d)
for f in cv_kernels cv_egress; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -x hip "$ROOT/cilium_amd/csrc/$f.hip" \
      -o "$T/$f.o" -Rpass-analysis=kernel-resource-usage 2>&1 \
  | sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' \
  | awk '/Function Name:/ {if (n) print n, v, s, o, l; n=$3; v=s=o=l=""}
         /VGPRs:/ && !/AGPR/ {v="vgpr=" $2} /ScratchSize/ {s="scratch=" $NF} /Occupancy/ {o="waves/SIMD=" $NF}
         /LDS Size/ {l="lds=" $NF} END {print n, v, s, o, l}'
done | c++filt | sed 's/(cv::[^)]*)//'
rm -rf "$T"
