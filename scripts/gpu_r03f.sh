#!/bin/bash
# Sintel B=1 / B=8 rocprof kernel stats of the product library (per-kernel split of the build)
set -u
bash scripts/gpu_profile.sh r03f/sintel sintel_b1_f32 || exit $?
bash scripts/gpu_profile.sh r03f/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
