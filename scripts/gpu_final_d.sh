#!/bin/bash
# KITTI NCHW (pack pass + DMA build) and channels-last (DMA build alone) on one box
set -u
R=${1:-r03}
bash scripts/gpu_profile.sh ${R}_d/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh ${R}_d/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
echo "== D done"
