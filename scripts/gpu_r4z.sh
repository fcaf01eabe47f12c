#!/bin/bash
# Round-4 session Z: epilogue pooling by v_permlane32_swap and select fixes (no
# spill in the f32 DMA build) — build tests, same-process A/B vs the previous
# library (bit identity asserted), Sintel bench.
set -u
O=gpurun_out/${RUN_TAG:-r4z}
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_channels_last.py tests/test_e2e_flow.py -x -q --timeout 300 --timeout-method thread
step ab_f32 400 python -u scripts/ab_build.py --shapes 1x55x128 8x55x128 1x46x62 --variants ws prev
step ab_bf16 300 python -u scripts/ab_build.py --dtype bf16 --shapes 8x47x156 --variants ws prev --layout nhwc
step bench 300 python -u bench.py --no-cpu-baseline
echo "== done"
