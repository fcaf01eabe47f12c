#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, no tracing domains)
# over an arbitrary command.  Usage:
#   bash scripts/gpu_pmc.sh <tag> <kernel regex> <command...>
# Output: gpurun_out/<tag>/p<i>.csv (counter_collection) + p<i>.log
set -u
TAG=$1; KRE=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY" \
         "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  N=p${i}
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "$KRE" --output-format csv \
    -d "$PWD/$OUT/$N" -o run -- "$@" > "$OUT/$N.log" 2>&1
  rc=$?; echo "== pmc $N rc=$rc"; tail -n 1 "$OUT/$N.log"
  find "$OUT/$N" -name '*counter_collection.csv' -exec cp {} "$OUT/$N.csv" \;
  rm -rf "$OUT/$N"
  [ $rc -eq 0 ] || exit $rc
done
echo "== pmc done"
