#!/bin/bash
# A/B: streaming stores for the conntrack stages' scattered per-packet outputs
set -u
bash tools/ab_libs.sh r01y/ab_ntst "config3 config5" cilium_amd/_lib/libcilium_hip_plst.so cilium_amd/_lib/libcilium_hip_ntst.so || exit 1
bash tools/ab_libs.sh r01y/ab_ntst2 "config3 config5" cilium_amd/_lib/libcilium_hip_ntst.so cilium_amd/_lib/libcilium_hip_plst.so || exit 1
