#!/bin/bash
# Lookup 256x16 shape for one-round grids: tests + headline bench
set -u
bash scripts/gpu_tests.sh r03l || exit $?
bash scripts/gpu_quick.sh r03l_b "" "--workload sintel --steps 200 --warmup 20" "--workload chairs --steps 200 --warmup 20"
