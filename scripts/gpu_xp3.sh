#!/bin/bash
set -u
TAG=${1:-xp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
run bf16_kitti 240 python -u scripts/xp_build.py --dtype bf16 --B 8 --H 47 --W 156 --xp 0,1,2,4,5 --launches 4 --rounds 5 --check 0
run trace 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/tr" -o run -- python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
find "$OUT/tr" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/tr"
echo "== done"
