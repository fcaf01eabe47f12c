set -u
bash scripts/gpu_profile.sh r01_cfg/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh r01_cfg/kitti kitti_b8_bf16 --workload kitti --no-cpu-baseline || exit $?
bash scripts/gpu_profile.sh r01_cfg/chairs chairs_b1_f32 --workload chairs --no-cpu-baseline || exit $?
bash scripts/gpu_profile.sh r01_cfg/hd_alt 1080p_b1_f32 --workload 1080p --block alt --no-cpu-baseline || exit $?
timeout -k 10 300 python -u bench.py --workload 1080p --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r01_cfg/hd_corr.log 2>&1; echo "hd corr rc=$?"; tail -1 gpurun_out/r01_cfg/hd_corr.log
