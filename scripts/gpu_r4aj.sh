#!/bin/bash
# Null A/B (-3 = an identical copy of this tree's library) beside the priority
# A/B (-3 = the same source without the lookup's level priority), Sintel and
# Chairs B=1, twice each: how large is the harness's own -1/-3 bias?
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for w in sintel chairs; do
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_same.so > gpurun_out/r4aj_${w}_null_$rep.json
  timeout -k 10 200 python -u scripts/ab_step.py --workload $w --variants -1 -3 --prev-lib scripts/libdexiraft_corr_noprio.so > gpurun_out/r4aj_${w}_noprio_$rep.json
done
done
