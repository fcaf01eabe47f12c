#!/bin/bash
# Round-4 refresh, part 2 of 2: B=8, 1080p (both blocks), training step, and the
# driver's own bench command.
set -u
R=r04
bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $?
mkdir -p gpurun_out/$R/backward
timeout -k 10 200 python -u scripts/time_backward.py --workload sintel > gpurun_out/$R/backward/time_backward_sintel.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/time_backward.py --workload chairs > gpurun_out/$R/backward/time_backward_chairs.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_driver_cmd.log 2>&1 || exit $?
echo "== part 2 done"
