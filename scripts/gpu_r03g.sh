#!/bin/bash
# Build and lookup ablations + timelines (experiments target)
set -u
O=gpurun_out/r03g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --trace > $O/xp_lookup_b1.log 2>&1; rc=$?; echo "xp b1 rc=$rc"; grep '^{' $O/xp_lookup_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 --trace > $O/xp_lookup_b8.log 2>&1; rc=$?; echo "xp b8 rc=$rc"; grep '^{' $O/xp_lookup_b8.log; exit $rc
