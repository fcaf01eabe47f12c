#!/bin/bash
set -u
bash scripts/gpu_pmc.sh r03d_pmc_b1 "corr_build_dma|split_pairs" python -u scripts/ab_build.py --variants ws --shapes 1x55x128 --reps 5 --rounds 1 || exit $?
bash scripts/gpu_pmc.sh r03d_pmc_b8 "corr_build_dma|split_pairs" python -u scripts/ab_build.py --variants ws --shapes 8x55x128 --reps 2 --rounds 1 || exit $?
python scripts/pmc_summary.py gpurun_out/r03d_pmc_b1 > gpurun_out/r03d_pmc_b1/summary.json
python scripts/pmc_summary.py gpurun_out/r03d_pmc_b8 > gpurun_out/r03d_pmc_b8/summary.json
