#!/bin/bash
# Ordered on-the-fly lookup: cell-load prefetch depth 1 / 2 / 4 (in-step)
set -u
O=gpurun_out/r03s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_step.py --workload 1080p --block alt --variants 100 102 103 --reps 5 > $O/ab_hd.log 2>&1; rc=$?; echo "ab rc=$rc"; grep '^{' $O/ab_hd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --block alt --variants 100 102 103 --reps 20 > $O/ab_sintel.log 2>&1; rc=$?; echo "ab sintel rc=$rc"; grep '^{' $O/ab_sintel.log
