#!/bin/bash
# Round-4 session G: half units last in every XCD's range (build order), tests + A/B
set -u
O=gpurun_out/r4g
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step ab_build 300 python -u scripts/ab_build.py --shapes 1x55x128 8x55x128 1x46x62 1x136x240 --variants ws prev --reps 10 --rounds 9
bash scripts/gpu_tests.sh r4g || exit $?
echo "== done"
