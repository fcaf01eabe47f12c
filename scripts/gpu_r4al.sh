#!/bin/bash
# Box check after a slow profile box: whole-build A/B (split PX 32 vs prev3's 64)
# with rocprofv3 kernel stats, then the Sintel profile again.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
P=scripts/libdexiraft_corr_prev3.so
timeout -k 10 300 python -u scripts/ab_build.py --variants ws prev --prev-lib $P --rounds 11 --shapes 1x55x128 1x46x62 > gpurun_out/r4al_build.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4al_prof" -o run -- python -u scripts/ab_build.py --variants prev --prev-lib $P --shapes 1x55x128 > gpurun_out/r4al_prof.log 2>&1
find gpurun_out/r4al_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4al_kernel_stats_prev.csv \;
rm -rf gpurun_out/r4al_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4al_prof" -o run -- python -u scripts/ab_build.py --variants ws --shapes 1x55x128 > gpurun_out/r4al_prof2.log 2>&1
find gpurun_out/r4al_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4al_kernel_stats_ws.csv \;
rm -rf gpurun_out/r4al_prof
bash scripts/gpu_profile.sh r04b/sintel sintel_b1_f32
