#!/bin/bash
# Round-4 session Y: hardware bf16 conversion in the build epilogue — bf16 tests,
# same-process A/B against the previous library (bit identity asserted), step A/B.
set -u
O=gpurun_out/r4y
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_bf16 500 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_channels_last.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bf16 or c3 or kitti or nhwc or channels"
step ab_kitti 300 python -u scripts/ab_build.py --dtype bf16 --shapes 8x47x156 1x55x128 --variants ws prev --layout nhwc
step ab_kitti_nchw 300 python -u scripts/ab_build.py --dtype bf16 --shapes 8x47x156 --variants ws prev
step bench_kitti 300 python -u bench.py --workload kitti --layout nhwc --no-cpu-baseline
echo "== done"
