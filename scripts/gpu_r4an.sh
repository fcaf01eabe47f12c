#!/bin/bash
# Last check of this round's library (GPU suite + smoke), then the 128 x 8
# lookup shape A/B (needs the experiments library).
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu_final.log 2>&1
tail -n 1 gpurun_out/r04/pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke_final.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/ab_step.py --workload sintel --variants -1 64 65 > gpurun_out/r4am_sintel_$rep.json
  timeout -k 10 200 python -u scripts/ab_step.py --workload chairs --variants -1 64 65 > gpurun_out/r4am_chairs_$rep.json
done
