#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash scripts/gpu_check.sh <tag> [bench args...]
# Each step has its own time limit; a step that faults, aborts, segfaults or
# times out (exit not in {0, 1}) ends the session — nothing else touches the GPU.
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
  tail -n 12 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)"
    exit "$rc"
  fi
  return 0
}

run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider
run bench 300 python -u bench.py --steps 30 --warmup 3 --cpu-seconds 8 "$@"
run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
  python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@"
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
rm -rf "$OUT/prof"
run e2e 300 python -u scripts/bench_e2e.py --workload chairs
echo "== done"
