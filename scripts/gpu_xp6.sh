set -u
mkdir -p gpurun_out/xp6
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_lookup.py --xp 0,1,2,4,8,16384 --check 8 --rounds 9 > gpurun_out/xp6/b1.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --xp 0,1,2,4,8 --rounds 9 > gpurun_out/xp6/b8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,1003:8,1003:16384 --rounds 7 > gpurun_out/xp6/step.log 2>&1 || exit $?
grep -h xp gpurun_out/xp6/*.log
