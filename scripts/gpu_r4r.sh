#!/bin/bash
# Round-4 session R: wave priority in the f32 DMA build (experiments XP 1024 / 2048).
set -u
O=gpurun_out/r4r
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step prio_sintel 300 python -u scripts/xp_build.py --xp 0 1024 2048 --split --trace-xp --rounds 7
step prio_b8 300 python -u scripts/xp_build.py --shape 8x55x128 --xp 0 1024 2048 --split --trace-xp --rounds 5
echo "== done"
