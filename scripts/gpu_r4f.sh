#!/bin/bash
# Round-4 session F: unrolled branch-free lookup phase 2 (product) against the
# previous product library (scripts/libdexiraft_corr_prev.so), in the step.
set -u
O=gpurun_out/r4f
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step parity_lookup 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step ab_sintel 200 python -u scripts/ab_step.py --workload sintel --variants -1 -3 --reps 50 --rounds 9
step ab_chairs 200 python -u scripts/ab_step.py --workload chairs --variants -1 -3 --reps 50 --rounds 9
step ab_sintel_b8 200 python -u scripts/ab_step.py --workload sintel --batch 8 --variants -1 -3 --reps 10 --rounds 7
step ab_kitti 200 python -u scripts/ab_step.py --workload kitti --batch 8 --dtype bf16 --variants -1 -3 --reps 10 --rounds 7
echo "== done"
