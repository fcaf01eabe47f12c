#!/bin/bash
# Round-4 experiment session B: the software-pipelined build.
set -u
O=gpurun_out/r4b
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step pipe_sintel 180 python -u scripts/xp_pipe.py --shape 1x55x128 --step
step pipe_sintel_b8 180 python -u scripts/xp_pipe.py --shape 8x55x128
step pipe_chairs 180 python -u scripts/xp_pipe.py --shape 1x46x62 --step
step pipe_kitti 180 python -u scripts/xp_pipe.py --shape 8x47x156 --dtype bf16
step pipe_odd 180 python -u scripts/xp_pipe.py --shape 2x30x44
echo "== done"
