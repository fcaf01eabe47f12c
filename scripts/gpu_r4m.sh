#!/bin/bash
# Round-4 session M: vectorised lookup-backward column pass — tests + same-process A/B.
set -u
O=gpurun_out/${RUN_TAG:-r4m}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_bw 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step ab_sintel 200 python -u scripts/ab_lookup_bw.py
step ab_chairs 200 python -u scripts/ab_lookup_bw.py --shape 1 46 62
step ab_b2r3 200 python -u scripts/ab_lookup_bw.py --shape 2 30 44 --radius 3
step tb_sintel 300 python -u scripts/time_backward.py --workload sintel
step tb_chairs 300 python -u scripts/time_backward.py --workload chairs
echo "== done"
