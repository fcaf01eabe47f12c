#!/bin/bash
# Round-3: build A/B with the parallel split pass, build ablations + timeline.
set -u
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_build.py --shapes 1x55x128 8x55x128 1x46x62 > $O/ab_build.log 2>&1; rc=$?; echo "ab_build rc=$rc"; grep '^{' $O/ab_build.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_ab" -o run -- python -u scripts/ab_build.py --shapes 1x55x128 1x46x62 --rounds 3 --variants ws > $O/ab_build_prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/prof_ab -name '*kernel_stats.csv' -exec cp {} $O/ab_kernel_stats.csv \; ; rm -rf $O/prof_ab
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/xp_build.py --shape 8x55x128 --reps 5 > $O/xp_build_b8.log 2>&1; rc=$?; echo "xp_build b8 rc=$rc"; grep '^{' $O/xp_build_b8.log; exit $rc
