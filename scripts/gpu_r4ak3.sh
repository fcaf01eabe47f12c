#!/bin/bash
# Split pass PX = 32 vs 64: whole-build A/B twice, then the same under rocprofv3
# kernel stats (split kernels are told apart by their PX template argument).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
P=scripts/libdexiraft_corr_prev3.so
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/ab_build.py --variants ws prev --prev-lib $P --rounds 11 --shapes 1x55x128 1x46x62 8x55x128 > gpurun_out/r4ak3_build_$rep.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4ak3_prof" -o run -- python -u scripts/ab_build.py --variants ws prev --prev-lib $P --shapes 1x55x128 > gpurun_out/r4ak3_prof.log 2>&1
find gpurun_out/r4ak3_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4ak3_kernel_stats.csv \;
rm -rf gpurun_out/r4ak3_prof
