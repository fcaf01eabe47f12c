#!/bin/bash
# Round-4 end session: smoke + full GPU suite, then bench + rocprofv3 kernel
# stats + FETCH/WRITE passes per BASELINE config (scripts/gpu_profile.sh),
# then the training-step timing.
set -u
R=${1:-r04}
bash scripts/gpu_tests.sh $R || exit $?
bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh $R/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $?
mkdir -p gpurun_out/$R/backward
timeout -k 10 200 python -u scripts/time_backward.py --workload sintel > gpurun_out/$R/backward/time_backward_sintel.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/time_backward.py --workload chairs > gpurun_out/$R/backward/time_backward_chairs.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_driver_cmd.log 2>&1 || exit $?
echo "== final done"
