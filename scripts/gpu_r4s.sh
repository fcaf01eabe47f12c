#!/bin/bash
# Round-4 session S: backward through other level counts; rocprofv3 kernel stats
# of the Sintel training step.
set -u
O=gpurun_out/r4s
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step tests_lv 300 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 200 --timeout-method thread -k "other_levels"
step prof_train 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python3 -u scripts/time_backward.py --workload sintel --reps 5
find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/train_kernel_stats.csv" \;
rm -rf "$O/prof"
echo "== done"
