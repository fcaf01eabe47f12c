#!/bin/bash
# PMC passes on the lookup (product kernel via scripts/xp_lookup.py variant 0), one counter group per run.
# Usage: bash scripts/gpu_pmc_lookup.sh <tag> [--B 8 ...]
set -u
TAG=${1:-pmc_lookup}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  N=p${i}
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "corr_lookup_wide" --output-format csv \
    -d "$PWD/$OUT/$N" -o run -- python -u scripts/xp_lookup.py --xp 0 --rounds 1 "$@" > "$OUT/$N.log" 2>&1
  rc=$?; echo "== pmc $N rc=$rc"; tail -n 1 "$OUT/$N.log"
  find "$OUT/$N" -name '*counter_collection.csv' -exec cp {} "$OUT/$N.csv" \;
  rm -rf "$OUT/$N"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "== done"
