#!/bin/bash
# Split-pass variants, lookup query-major gathers on levels 2/3
set -u
O=gpurun_out/r03i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 --xp 0 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/xp_build.py --shape 8x55x128 --xp 0 --reps 5 > $O/xp_build_b8.log 2>&1; rc=$?; echo "xp_build b8 rc=$rc"; grep '^{' $O/xp_build_b8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --trace > $O/xp_lookup_b1.log 2>&1; rc=$?; echo "xp b1 rc=$rc"; grep '^{' $O/xp_lookup_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 --trace > $O/xp_lookup_b8.log 2>&1; rc=$?; echo "xp b8 rc=$rc"; grep '^{' $O/xp_lookup_b8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 --hw 47 156 --dtype bf16 --xp 0 32 > $O/xp_lookup_kitti.log 2>&1; rc=$?; echo "xp kitti rc=$rc"; grep '^{' $O/xp_lookup_kitti.log; exit $rc
