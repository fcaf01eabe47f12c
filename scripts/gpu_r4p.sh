#!/bin/bash
# Round-4 session P: training-path host changes (no token gradients, side-stream
# zero fill of the gradient pyramid) — backward tests + training-step timing.
set -u
O=gpurun_out/${RUN_TAG:-r4p}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_bw 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py tests/test_e2e_flow.py -x -q --timeout 300 --timeout-method thread
step tb_sintel 300 python -u scripts/time_backward.py --workload sintel
step tb_chairs 300 python -u scripts/time_backward.py --workload chairs
step tb_sintel2 300 python -u scripts/time_backward.py --workload sintel --reps 30
echo "== done"
