#!/bin/bash
# Round-3: inline non-finite fallback + write-through split pass: tests, A/B, benches
set -u
bash scripts/gpu_tests.sh r03h || exit $?
O=gpurun_out/r03h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/xp_build.py --shape 1x55x128 > $O/xp_build_b1.log 2>&1; rc=$?; echo "xp_build b1 rc=$rc"; grep '^{' $O/xp_build_b1.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_quick.sh r03h_b "" "--workload sintel --steps 200 --warmup 20" "--workload sintel --batch 8" "--workload chairs --steps 200 --warmup 20"
