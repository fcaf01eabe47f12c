#!/bin/bash
# Lookup shape at B=1: 128 threads x 8 queries (65) vs the product's 256 x 16
# (-1, and 64 = the same shape through the experiments library), in the step.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --variants -1 64 65 > gpurun_out/r4am_sintel_$rep.json
  timeout -k 10 200 python -u scripts/ab_step.py --workload chairs --variants -1 64 65 > gpurun_out/r4am_chairs_$rep.json
done
