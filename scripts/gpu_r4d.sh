#!/bin/bash
# Round-4 experiment session D: desynchronising the two workgroups of a CU in
# the DMA build (round-1 second-slot delay), co-residence of the first round.
set -u
O=gpurun_out/r4d
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 6 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step build_delay 240 python -u scripts/xp_build.py --shape 1x55x128 --xp 0 16896 33280 49664 66048 --split --trace-xp 256 33536 49920
step build_delay_b8 240 python -u scripts/xp_build.py --shape 8x55x128 --xp 0 33280 49664 --split --trace-xp
echo "== done"
