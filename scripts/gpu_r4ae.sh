#!/bin/bash
# Same-process A/B in the bench's step: lookup with the coarsest level dispatched
# first (-1, this tree) vs the previous library's lookup (-3).
set -e
mkdir -p gpurun_out
P=scripts/libdexiraft_corr_prev3.so
timeout -k 10 150 python -u scripts/ab_step.py --workload sintel --variants -1 -3 --prev-lib $P > gpurun_out/r4ae_sintel.json
timeout -k 10 150 python -u scripts/ab_step.py --workload chairs --variants -1 -3 --prev-lib $P > gpurun_out/r4ae_chairs.json
timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --batch 8 --variants -1 -3 --prev-lib $P > gpurun_out/r4ae_sintel_b8.json
timeout -k 10 200 python -u scripts/ab_step.py --workload kitti --batch 8 --dtype bf16 --variants -1 -3 --prev-lib $P > gpurun_out/r4ae_kitti.json
