#!/bin/bash
# Chunk 0 of the fmap-gradient GEMMs sums into the output: backward tests, then
# the Sintel / Chairs training step (time and peak memory).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_backward.py > gpurun_out/r4ah_tests.log 2>&1
timeout -k 10 200 python -u scripts/time_backward.py --workload sintel > gpurun_out/r4ah_time_sintel.json
timeout -k 10 200 python -u scripts/time_backward.py --workload chairs > gpurun_out/r4ah_time_chairs.json
