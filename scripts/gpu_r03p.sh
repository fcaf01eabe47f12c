#!/bin/bash
# Parallel query ordering for the on-the-fly lookup: alt tests, in-step A/B, kernel times
set -u
O=gpurun_out/r03p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "alt or alternate or c5 or smoke" > $O/pytest_alt.log 2>&1; rc=$?; echo "pytest alt rc=$rc"; tail -2 $O/pytest_alt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_step.py --workload 1080p --block alt --variants -1 -2 --reps 5 > $O/ab_hd.log 2>&1; rc=$?; echo "ab rc=$rc"; grep '^{' $O/ab_hd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --block alt --variants -1 -2 --reps 20 > $O/ab_sintel.log 2>&1; rc=$?; echo "ab sintel rc=$rc"; grep '^{' $O/ab_sintel.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/p" -o run -- python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 --reps 5 --rounds 3 > $O/p.log 2>&1; rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/p -name '*kernel_stats.csv' -exec cp {} $O/stats.csv \; ; rm -rf $O/p
