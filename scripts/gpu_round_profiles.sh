#!/bin/bash
# All round profiles in one GPU call: scripts/gpu_profile.sh for each BASELINE
# config (bench line, rocprofv3 kernel stats, FETCH/WRITE PMC passes), outputs
# under gpurun_out/<round>/<config>.  Stops at the first failing session.
# Usage: bash scripts/gpu_round_profiles.sh <round tag, e.g. r03>
set -u
R=${1:-r03}
bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh $R/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $?
echo "== all done"
