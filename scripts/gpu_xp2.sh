#!/bin/bash
# Split-build timing after a change: xp ablations (Sintel B=1, B=8) + GPU parity of the build.
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
  tail -n 14 "$OUT/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "== stopping after $name (rc=$rc)"; exit "$rc"; fi
  return 0
}
run xp_sintel 240 python -u scripts/xp_build.py --xp ${XPS:-0,1,2,4,5,8} --check ${CHECK:-0}
run xp_b8 240 python -u scripts/xp_build.py --B 8 --xp ${XPB8:-0,1} --launches 4 --rounds 5
[ -n "${SKIP_PYTEST:-}" ] || run pytest_build 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_channels_last.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
echo "== done"
