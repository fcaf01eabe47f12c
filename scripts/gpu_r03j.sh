#!/bin/bash
# bf16 LDS-DMA build, whole-line split stores, query-major lookup gathers: tests + A/B + benches
set -u
bash scripts/gpu_tests.sh r03j || exit $?
O=gpurun_out/r03j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 --xp 0 32 --split 0 1 4 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/xp_build.py --shape 8x55x128 --xp 0 32 --split 0 1 4 --reps 5 > $O/xp_build_b8.log 2>&1; rc=$?; echo "xp_build b8 rc=$rc"; grep '^{' $O/xp_build_b8.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_quick.sh r03j_b "" "--workload sintel --steps 200 --warmup 20" "--workload kitti --steps 100" "--workload kitti --layout nhwc --steps 100" "--workload sintel --batch 8 --steps 100"
