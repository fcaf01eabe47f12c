#!/bin/bash
# PMC counter passes for the correlation kernels (one rocprofv3 run per pass;
# never combined with tracing domains).  Usage: bash scripts/profile_pmc.sh <tag> [bench args]
# Output: gpurun_out/<tag>/pmc/<pass>/..._counter_collection.csv
set -u
TAG=${1:-pmc}
shift || true
OUT=$PWD/gpurun_out/$TAG/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python -u bench.py --steps 4 --warmup 1 --mode eager --no-cpu-baseline "$@")

timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
echo "counter list rc=$?"

pass() {  # name counters...
  local name=$1
  shift
  mkdir -p "$OUT/$name"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "corr_|alt_corr|avg_pool" \
    --output-format csv -d "$OUT/$name" -o run -- "${BENCH[@]}" > "$OUT/$name/log.txt" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  tail -n 3 "$OUT/$name/log.txt"
  if [ "$rc" -ne 0 ]; then exit "$rc"; fi
}

pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT \
  SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM
pass fetch FETCH_SIZE TCC_HIT_sum
pass write WRITE_SIZE TCC_MISS_sum TCC_EA0_WRREQ_64B_sum
echo "== pmc done"
