#!/bin/bash
# Confirm: level priority on the one-round lookup shape only (-1) vs prev3 (-3).
set -e
mkdir -p gpurun_out
for w in "sintel --batch 1" "chairs --batch 1" "sintel --batch 8" "kitti --batch 1 --dtype bf16"; do
  n=$(echo $w | tr -d ' -')
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_prev3.so > gpurun_out/r4ag_${n}.json
done
