set -u
mkdir -p gpurun_out/xp16
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_trace.py > gpurun_out/xp16/trace.log 2>&1 || exit $?
cat gpurun_out/xp16/trace.log | cut -c1-1500
