#!/bin/bash
# Lookup ablations/variants (experiments lib) at B=1, B=8 f32, KITTI B=8 bf16, + PMC traffic at B=8.
set -u
TAG=${1:-xpl}
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
X=${XPL:-0,1,2,3,4}
C=${CHECKL:-}
run b1 200 python -u scripts/xp_lookup.py --xp $X ${C:+--check $C}
run b8 200 python -u scripts/xp_lookup.py --B 8 --xp $X ${C:+--check $C}
run kitti8 200 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp ${XPLB:-0,1,2} ${C:+--check $C}
if [ -n "${PMCL:-}" ]; then
for CNT in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $CNT --kernel-include-regex "corr_lookup" --output-format csv \
    -d "$PWD/$OUT/pmc_$CNT" -o run -- python -u scripts/xp_lookup.py --B 8 --xp $PMCL --rounds 1 > "$OUT/pmc_$CNT.log" 2>&1
  rc=$?; echo "== pmc $CNT rc=$rc"
  find "$OUT/pmc_$CNT" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_$CNT.csv" \;
  rm -rf "$OUT/pmc_$CNT"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
fi
echo "== done"
