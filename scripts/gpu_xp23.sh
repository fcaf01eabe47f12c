set -u
mkdir -p gpurun_out/xp23
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_build.py --xp 1003,4500 --check 4500 --ref 1003 --rounds 3 > gpurun_out/xp23/chk.log 2>&1 || exit $?
grep -h "bit" gpurun_out/xp23/chk.log
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,4500 --rounds 11 > gpurun_out/xp23/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,4500 --rounds 5 > gpurun_out/xp23/sintel8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_accuracy.py > gpurun_out/xp23/acc.log 2>&1; tail -3 gpurun_out/xp23/acc.log
grep -h "xp" gpurun_out/xp23/sintel*.log
