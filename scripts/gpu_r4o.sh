#!/bin/bash
# Round-4 session O: single-launch query ordering of the on-the-fly lookup —
# parity (bit-identity of the orders, configs) + same-process A/B vs the
# three-launch ordering (experiments variant 109).
set -u
O=gpurun_out/${RUN_TAG:-r4o}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_alt 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_channels_last.py -x -q --timeout 300 --timeout-method thread -k "alt or Alternate or c5 or 1080"
step ab_hd 300 python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 109 --reps 5 --rounds 7
step ab_sintel 300 python -u scripts/ab_step.py --workload sintel --block alt --variants -2 109 --reps 10 --rounds 7
echo "== done"
