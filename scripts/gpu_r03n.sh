#!/bin/bash
# In-step A/B: lookup shapes (Sintel B=1/B=8, Chairs, KITTI bf16) and ordered on-the-fly lookups (1080p)
set -u
O=gpurun_out/r03n; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 200 python -u scripts/ab_step.py "$@" > $O/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; grep '^{' $O/$n.log; [ $rc -eq 0 ] || exit $rc; }
run sintel --workload sintel --variants -1 32 64 0
run chairs --workload chairs --variants -1 32 64
run sintel_b8 --workload sintel --batch 8 --variants -1 32 64 --reps 10
run kitti --workload kitti --batch 8 --dtype bf16 --variants -1 32 64 --reps 10
run hd_alt --workload 1080p --block alt --variants -1 -2 --reps 5
