#!/bin/bash
# Round-4 session H: PMC passes over the f32 DMA build and the wide lookup (Sintel).
set -u
bash scripts/gpu_pmc.sh pmc_build "corr_build_dma|corr_lookup_wide|split_pairs" \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline --clock-warmup-s 0.1
