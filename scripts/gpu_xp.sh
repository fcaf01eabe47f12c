#!/bin/bash
# Experiments session (via gpurun, repo root): split-build ablations and PMC
# counter passes on the build kernel.  Usage: bash scripts/gpu_xp.sh <tag>
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
run xp_sintel 240 python -u scripts/xp_build.py --xp 0,1,2,4,5,8,16,3,19
run xp_b8 240 python -u scripts/xp_build.py --B 8 --xp 0,1,2,4,8 --launches 4 --rounds 5
run counters 60 rocprofv3 -L
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "corr_build_split" --output-format csv \
    -d "$PWD/$OUT/pmc_$N" -o run -- python -u scripts/xp_build.py --xp 0 --launches 2 --rounds 2 > "$OUT/pmc_$N.log" 2>&1
  rc=$?; echo "== pmc $N rc=$rc"; tail -n 3 "$OUT/pmc_$N.log"
  find "$OUT/pmc_$N" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_$N.csv" \;
  rm -rf "$OUT/pmc_$N"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "== done"
