#!/bin/bash
# PMC pass over the training step (scripts/time_backward.py): stall profile of
# corr_lookup_backward_kernel and fmap_grad_kernel.  Outputs gpurun_out/pmclb/.
export TMPDIR=/tmp
OUT=gpurun_out/pmclb
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM -d $OUT/p1 -o p1 -- python3 scripts/time_backward.py --reps 2 > $OUT/p1.log 2>&1 || exit 1
echo skip-p2
echo done
