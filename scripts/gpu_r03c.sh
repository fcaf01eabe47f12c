#!/bin/bash
# Round-3: full GPU tests, build A/B, build ablations + timeline, benches.
set -u
bash scripts/gpu_tests.sh r03c || exit $?
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_build.py --shapes 1x55x128 8x55x128 1x46x62 8x47x156 > $O/ab_build.log 2>&1; rc=$?; echo "ab_build rc=$rc"; grep '^{' $O/ab_build.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/xp_build.py --shape 8x55x128 --reps 5 > $O/xp_build_b8.log 2>&1; rc=$?; echo "xp_build b8 rc=$rc"; grep '^{' $O/xp_build_b8.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_quick.sh r03c_b "" "--workload sintel" "--workload chairs" "--workload sintel --batch 8"
