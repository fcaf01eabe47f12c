#!/bin/bash
# Step-level A/B of the 32-pixel split pass (-1) vs prev3 (-3), twice each on
# Sintel and Chairs, a null A/B beside it; then the parity tests.
set -e
mkdir -p gpurun_out
P=scripts/libdexiraft_corr_prev3.so
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --variants -1 -3 --prev-lib $P > gpurun_out/r4ak_step_sintel_$rep.json
  timeout -k 10 200 python -u scripts/ab_step.py --workload chairs --variants -1 -3 --prev-lib $P > gpurun_out/r4ak_step_chairs_$rep.json
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_channels_last.py > gpurun_out/r4ak_tests.log 2>&1
