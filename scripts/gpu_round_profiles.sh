#!/bin/bash
# All round profiles in one GPU call: scripts/gpu_profile.sh for each BASELINE
# config (bench line, rocprofv3 kernel stats, FETCH/WRITE PMC passes).
# Stops at the first failing session.
set -u
bash scripts/gpu_profile.sh p_sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh p_chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh p_kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh p_hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
echo "== all done"
