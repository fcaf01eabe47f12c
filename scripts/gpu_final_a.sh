#!/bin/bash
# Round-end session A: smoke + full GPU suite, then profiles of Sintel / Chairs / KITTI (NCHW, NHWC)
set -u
R=${1:-r03}
bash scripts/gpu_tests.sh $R || exit $?
bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh $R/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
echo "== A done"
