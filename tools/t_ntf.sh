#!/bin/bash
# A/B: streaming stores for k_netdev_front's per-packet scratch and outputs (config 3)
set -u
bash tools/ab_libs.sh r01z/ab_ntf config3 cilium_amd/_lib/libcilium_hip_plf.so cilium_amd/_lib/libcilium_hip_ntf.so || exit 1
bash tools/ab_libs.sh r01z/ab_ntf2 config3 cilium_amd/_lib/libcilium_hip_ntf.so cilium_amd/_lib/libcilium_hip_plf.so || exit 1
bash tools/ab_libs.sh r01z/ab_ntf3 config3 cilium_amd/_lib/libcilium_hip_plf.so cilium_amd/_lib/libcilium_hip_ntf.so || exit 1
