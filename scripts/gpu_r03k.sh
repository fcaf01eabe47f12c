#!/bin/bash
# Lookup workgroup shapes (256 x 16 / 512 x 32 / 1024 x 64)
set -u
O=gpurun_out/r03k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/xp_lookup.py > $O/xp_lookup_b1.log 2>&1; rc=$?; echo "xp b1 rc=$rc"; grep '^{' $O/xp_lookup_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 > $O/xp_lookup_b8.log 2>&1; rc=$?; echo "xp b8 rc=$rc"; grep '^{' $O/xp_lookup_b8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --hw 46 62 > $O/xp_lookup_chairs.log 2>&1; rc=$?; echo "xp chairs rc=$rc"; grep '^{' $O/xp_lookup_chairs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 --hw 47 156 --dtype bf16 --xp 0 32 64 128 > $O/xp_lookup_kitti.log 2>&1; rc=$?; echo "xp kitti rc=$rc"; grep '^{' $O/xp_lookup_kitti.log; exit $rc
