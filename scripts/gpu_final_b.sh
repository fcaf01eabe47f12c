#!/bin/bash
# Round-end session B: profiles of Sintel B=8 and 1080p (on the fly, full pyramid)
set -u
R=${1:-r03}
bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $?
echo "== B done"
