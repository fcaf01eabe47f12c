set -u
mkdir -p gpurun_out/xp22
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_build.py --xp 1003,4400,4401,4402 --check 4400,4401,4402 --ref 1003 --rounds 3 > gpurun_out/xp22/chk.log 2>&1 || exit $?
grep -h "bit\|xp" gpurun_out/xp22/chk.log
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,4400,4401,4402 --rounds 9 > gpurun_out/xp22/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,4402 --rounds 5 > gpurun_out/xp22/sintel8.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp22/sintel*.log
