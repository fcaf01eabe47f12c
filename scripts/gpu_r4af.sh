#!/bin/bash
# Same-process A/Bs in the bench's step: lookup wave priority by level.
# -1 = this tree (prio 3/2/1/0 by level), -3 = --prev-lib (prev3: no priority;
# xA: level 0 only at priority 3).
set -e
mkdir -p gpurun_out
for w in "sintel --batch 1" "chairs --batch 1" "sintel --batch 8" "kitti --batch 8 --dtype bf16"; do
  n=$(echo $w | tr -d ' -')
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_prev3.so > gpurun_out/r4af_${n}_base.json
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_xA.so > gpurun_out/r4af_${n}_xA.json
done
