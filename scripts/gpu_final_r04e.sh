#!/bin/bash
# Round-4 final checks after the split pass went to 32-pixel workgroups: the
# whole GPU suite, smoke, the profiles of every config whose build runs the
# split pass (Sintel B=1 / B=8, Chairs, 1080p full pyramid), the driver's command.
set -u
R=r04
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_gpu_final.log 2>&1 || exit $?
tail -n 2 gpurun_out/$R/pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke_final.log 2>&1 || exit $?
bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $?
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$R/bench_driver_cmd.log 2>&1 || exit $?
echo "== final done"
