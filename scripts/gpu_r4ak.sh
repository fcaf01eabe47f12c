#!/bin/bash
# Split pass at 32 pixels x 16 channel blocks per workgroup (512 threads, two per
# CU) vs 64 (prev3): whole builds, same process, bit-identity checked; then the
# split tests.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_build.py --variants ws prev --prev-lib scripts/libdexiraft_corr_prev3.so --shapes 1x55x128 8x55x128 1x46x62 > gpurun_out/r4ak_build.json
timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --variants -1 -3 --prev-lib scripts/libdexiraft_corr_prev3.so > gpurun_out/r4ak_step_sintel.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_channels_last.py > gpurun_out/r4ak_tests.log 2>&1
