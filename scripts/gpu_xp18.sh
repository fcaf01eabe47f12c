set -u
mkdir -p gpurun_out/xp18
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_build.py --xp 1003,4300,4301 --check 4300,4301 --ref 1003 --rounds 3 > gpurun_out/xp18/chk.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,4300,4301 --rounds 9 > gpurun_out/xp18/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,4301 --rounds 5 > gpurun_out/xp18/sintel8.log 2>&1 || exit $?
grep -h "xp\|bit" gpurun_out/xp18/*.log
