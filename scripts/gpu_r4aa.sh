#!/bin/bash
# Round-4 session AA: lookup gather addressing by shifts / 24-bit multiplies and
# pointer-stepped output stores — lookup tests + in-step A/B vs previous library.
set -u
O=gpurun_out/r4aa
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 2 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_motion.py tests/test_gpu_channels_last.py -x -q --timeout 300 --timeout-method thread
step ab_sintel 300 python -u scripts/ab_step.py --workload sintel --variants -1 -3 --reps 50 --rounds 9
step ab_chairs 300 python -u scripts/ab_step.py --workload chairs --variants -1 -3 --reps 50 --rounds 9
step ab_sintel_b8 300 python -u scripts/ab_step.py --workload sintel --batch 8 --variants -1 -3 --reps 10 --rounds 7
step ab_kitti 300 python -u scripts/ab_step.py --workload kitti --batch 8 --dtype bf16 --variants -1 -3 --reps 10 --rounds 7
echo "== done"
