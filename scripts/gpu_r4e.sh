#!/bin/bash
# Round-4 session E: the chained (in-kernel ordered) chunk reduction of the
# fused backward GEMMs: backward tests + training-step timing / memory.
set -u
O=gpurun_out/r4e
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_backward 400 python -u -m pytest tests/test_gpu_backward.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step time_bw_sintel 200 python -u scripts/time_backward.py --workload sintel
step time_bw_chairs 200 python -u scripts/time_backward.py --workload chairs
echo "== done"
