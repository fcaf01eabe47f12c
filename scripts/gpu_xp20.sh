set -u
mkdir -p gpurun_out/xp20
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "backward or training or grad" > gpurun_out/xp20/pytest_bw.log 2>&1; rc=$?; tail -2 gpurun_out/xp20/pytest_bw.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/time_backward.py --workload sintel > gpurun_out/xp20/bw_sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/time_backward.py --workload chairs > gpurun_out/xp20/bw_chairs.log 2>&1 || exit $?
grep -h "^{" gpurun_out/xp20/bw_*.log
