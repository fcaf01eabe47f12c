#!/bin/bash
# Multi-round lookup grids with levels interleaved along the dispatch order (-1)
# vs the level-major order (-3, prev3 = previous commit).
set -e
mkdir -p gpurun_out
for w in "sintel --batch 8" "kitti --batch 8 --dtype bf16" "1080p --batch 1" "sintel --batch 1"; do
  n=$(echo $w | tr -d ' -')
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_prev3.so > gpurun_out/r4ai_${n}.json
done
