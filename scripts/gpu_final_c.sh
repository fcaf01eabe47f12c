#!/bin/bash
# Round-end session C: bf16 pack pass with whole-line stores (tests + KITTI NCHW profile), 1080p on-the-fly trace
set -u
R=${1:-r03}
O=gpurun_out/$R; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "bf16 or kitti or c3 or capi" > $O/pytest_bf16.log 2>&1; rc=$?; echo "pytest bf16 rc=$rc"; tail -2 $O/pytest_bf16.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?

timeout -k 10 200 python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 103 104 105 --reps 5 > $O/ab_pf.log 2>&1; rc=$?; echo "ab pf rc=$rc"; grep '^{' $O/ab_pf.log
echo "== C done"
