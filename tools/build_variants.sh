#!/bin/bash
# A/B variants of the HIP library (timing only): how the egress conntrack stage walks
# its groups (CV_EG_RUNS, cilium_amd/csrc/cv_dp.hpp)
set -e
cd "$(dirname "$0")/.."
python -m cilium_amd.build -f
python - <<'PY'
from cilium_amd import build
L = "cilium_amd/_lib/"
for m in (0, 1, 3):
    build.build(True, out=L + f"libcilium_hip_eg{m}.so", defines=(f"CV_EG_RUNS={m}",))
PY
