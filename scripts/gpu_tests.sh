#!/bin/bash
# Smoke + the whole -m gpu suite (one process), logs under gpurun_out/<tag>.
set -u
OUT=gpurun_out/${1:-tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "== smoke rc=$rc"; tail -n 1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -n 2 "$OUT/pytest_gpu.log"; exit $rc
