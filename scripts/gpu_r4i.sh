#!/bin/bash
# Round-4 session I: the bounded (f16 pair) fmap-gradient GEMMs — parity tests,
# same-process A/B against the six-product form, training-step timing.
set -u
O=gpurun_out/${RUN_TAG:-r4i}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_bw 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
step ab_sintel 200 python -u scripts/ab_fmap_grads.py
step ab_chairs 200 python -u scripts/ab_fmap_grads.py --shape 1 256 46 62 4
step tb_sintel 300 python -u scripts/time_backward.py --workload sintel
step tb_chairs 300 python -u scripts/time_backward.py --workload chairs
echo "== done"
