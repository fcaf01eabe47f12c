#!/bin/bash
# End-of-round GPU call: smoke, the whole -m gpu suite, then the
# per-config profiles (bench + rocprof + trace timeline + FETCH/WRITE passes).
set -u
R=${1:-r03}
OUT=gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -n 1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -n 2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_round_profiles.sh "$R" > "$OUT/profiles.log" 2>&1
rc=$?; echo "== profiles rc=$rc"; tail -n 2 "$OUT/profiles.log"; exit $rc
