#!/bin/bash
# Channels-last session: new parity tests, the full GPU suite, and 1080p-alt /
# Sintel benches in both fmap layouts.  Each step has its own time limit; any
# failure ends the session.
set -u
O=gpurun_out/${1:-nhwc}
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?; echo "== $n rc=$rc"; tail -n 3 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step t_cl 300 python -u -m pytest tests/test_gpu_channels_last.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step t_all 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step b_alt_nchw 240 python -u bench.py --workload 1080p --block alt --steps 20 --warmup 3 --no-cpu-baseline
step b_alt_nhwc 240 python -u bench.py --workload 1080p --block alt --steps 20 --warmup 3 --no-cpu-baseline --layout nhwc
step b_sintel_nhwc 240 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --layout nhwc
step prof_alt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_alt" -o run -- python -u bench.py --workload 1080p --block alt --steps 20 --warmup 3 --no-cpu-baseline
find "$O/prof_alt" -name '*kernel_stats.csv' -exec cp {} "$O/alt_kernel_stats.csv" \;
rm -rf "$O/prof_alt"
echo "== done"
