#!/bin/bash
# On-the-fly lookup: LDS-DMA cell staging variant vs product (in-step), PMC of the product kernel
set -u
O=gpurun_out/r03r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 100 101 --reps 5 > $O/ab_hd.log 2>&1; rc=$?; echo "ab rc=$rc"; grep '^{' $O/ab_hd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --block alt --variants -2 101 --reps 20 > $O/ab_sintel.log 2>&1; rc=$?; echo "ab sintel rc=$rc"; grep '^{' $O/ab_sintel.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh r03r/pmc "alt_corr_mfma" python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 --reps 2 --rounds 1 || exit $?
python scripts/pmc_summary.py gpurun_out/r03r/pmc > gpurun_out/r03r/pmc/summary.json
