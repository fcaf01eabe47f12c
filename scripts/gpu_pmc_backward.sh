export TMPDIR=/tmp
mkdir -p gpurun_out/pmcbw
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pmcbw/pytest.log 2>&1 || { tail -5 gpurun_out/pmcbw/pytest.log; exit 1; }
tail -2 gpurun_out/pmcbw/pytest.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcbw/kt -o kt -- python3 scripts/xp_backward.py optical-flow_dexi-raft_amd/libdexiraft_corr.so --reps 10 > gpurun_out/pmcbw/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmcbw/p1 -o p1 -- python3 scripts/xp_backward.py optical-flow_dexi-raft_amd/libdexiraft_corr.so --reps 3 > gpurun_out/pmcbw/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmcbw/p2 -o p2 -- python3 scripts/xp_backward.py optical-flow_dexi-raft_amd/libdexiraft_corr.so --reps 3 > gpurun_out/pmcbw/p2.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/xp_backward.py xp_so/l1.so xp_so/l2.so > gpurun_out/pmcbw/ab.log 2>&1 && grep lib gpurun_out/pmcbw/ab.log
