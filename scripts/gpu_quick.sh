#!/bin/bash
# Quick GPU check after a kernel change: selected pytest, then bench lines.
# Usage: bash scripts/gpu_quick.sh <tag> "<pytest -k expr or empty>" "<bench args 1>" ["<bench args 2>" ...]
set -u
TAG=$1; K=$2; shift 2
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
  tail -n 6 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
if [ -n "$K" ]; then
  run pytest 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K"
fi
i=0
for A in "$@"; do
  i=$((i+1))
  run bench$i 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $A
done
echo "== done"
