#!/bin/bash
# Round-3 GPU session: tests, quick benches, lookup ablations + timeline.
set -u
bash scripts/gpu_tests.sh r03a || exit $?
bash scripts/gpu_quick.sh r03a_b "" "--workload sintel" "--workload sintel --layout nhwc" "--workload chairs" "--workload kitti" "--workload kitti --layout nhwc" "--workload sintel --batch 8" || exit $?
O=gpurun_out/r03a_xp; mkdir -p $O
timeout -k 10 120 python -u scripts/xp_lookup.py --trace > $O/xp_lookup_b1.log 2>&1; rc=$?; echo "xp b1 rc=$rc"; tail -5 $O/xp_lookup_b1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/xp_lookup.py --batch 8 --trace > $O/xp_lookup_b8.log 2>&1; rc=$?; echo "xp b8 rc=$rc"; tail -5 $O/xp_lookup_b8.log; exit $rc
