#!/bin/bash
# Short GPU-box session: smoke, GPU parity tests, bench (with CPU baseline), rocprofv3 stats.
# Usage (repo root, via gpurun): bash scripts/gpu_round.sh <tag> [bench args...]
set -u
TAG=${1:-dev}
shift || true
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
  tail -n 8 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
[ -z "${SKIP_TESTS:-}" ] && run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
[ -z "${SKIP_TESTS:-}" ] && run pytest_gpu 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run bench 240 python -u bench.py --steps 30 --warmup 3 --cpu-seconds 10 "$@"
run rocprof 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
  python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
echo "== done"
