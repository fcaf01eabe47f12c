#!/bin/bash
# Round profile session (via gpurun, repo root): bench line, rocprofv3 kernel
# stats of the same command, and FETCH_SIZE / WRITE_SIZE passes (one counter
# group per rocprofv3 run) -> traffic.json.
# Usage: bash scripts/gpu_profile.sh <tag> <workload key> [bench args...]
set -u
TAG=${1:-prof}
WKEY=${2:-sintel_b1_f32}
shift 2 || true
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --cpu-seconds 10 "$@" > "$O/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 "$O/bench.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o run -- \
  python -u bench.py --no-cpu-baseline "$@" > "$O/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;
grep '^{' "$O/prof.log" | tail -n 1 > "$O/bench_under_rocprof.json"
find "$O/prof" -name '*kernel_trace.csv' -exec python scripts/trace_gaps.py {} "$WKEY" \; > "$O/trace_gaps.json" 2>&1
rm -rf "$O/prof"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "corr_" --output-format csv \
    -d "$PWD/$O/pmc_$C" -o run -- python -u bench.py --steps 4 --warmup 1 --mode eager \
    --clock-warmup-s 0 --no-cpu-baseline "$@" > "$O/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find "$O/pmc_$C" -name '*counter_collection.csv' -exec cp {} "$O/pmc_$C.csv" \;
  rm -rf "$O/pmc_$C"
done
python scripts/pmc_traffic.py "$O/pmc_FETCH_SIZE.csv" "$O/pmc_WRITE_SIZE.csv" "$WKEY" "$TAG" > "$O/traffic.json"
echo "== done"
