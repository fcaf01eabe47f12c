#!/bin/bash
# Ordered alt lookup tests + 1080p alt bench; Sintel step profile (lookup shape check)
set -u
O=gpurun_out/r03m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "alt or alternate or c5" > $O/pytest_alt.log 2>&1; rc=$?; echo "pytest alt rc=$rc"; tail -2 $O/pytest_alt.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_quick.sh r03m_b "" "--workload 1080p --block alt" || exit $?
bash scripts/gpu_profile.sh r03m/sintel sintel_b1_f32
