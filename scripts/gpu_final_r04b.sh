#!/bin/bash
# Round-4 refresh after the epilogue changes, part 1 of 2: smoke + GPU suite,
# then the bench / rocprofv3 / traffic profile of four configs.
set -u
R=r04
bash scripts/gpu_tests.sh $R || exit $?
bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh $R/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
echo "== part 1 done"
