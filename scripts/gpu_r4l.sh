#!/bin/bash
# Round-4 session L: NaN-through-CorrBlock test of the bounded backward; on-the-fly
# lookup split ablation (experiments variant 108 = product without the cell split).
set -u
O=gpurun_out/r4l
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}

step alt_split 300 python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 103 108 --no-check 108 --reps 5 --rounds 5
echo "== done"
