#!/bin/bash
# Kernel times of the ordered vs tile-order on-the-fly lookup in the step
set -u
O=gpurun_out/r03o; mkdir -p $O
export TMPDIR=/tmp
for V in -1 -2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/p$V" -o run -- python -u scripts/ab_step.py --workload 1080p --block alt --variants $V --reps 5 --rounds 3 > $O/p$V.log 2>&1; rc=$?; echo "rocprof $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $O/p$V -name '*kernel_stats.csv' -exec cp {} $O/stats$V.csv \; ; rm -rf $O/p$V
done
