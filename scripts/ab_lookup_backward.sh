export TMPDIR=/tmp
mkdir -p gpurun_out/ablb
for v in c a b c a b; do
  cp xp_so/lb_$v.so optical-flow_dexi-raft_amd/libdexiraft_corr.so
  timeout -k 10 120 python -u scripts/time_backward.py --workload sintel > gpurun_out/ablb/$v.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ablb/$v.json').read().strip().splitlines()[-1]); print('$v', d['train_step_ms'], d['kernel_ms_one_step']['corr_lookup_backward'])"
done
