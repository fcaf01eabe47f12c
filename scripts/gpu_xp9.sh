set -u
mkdir -p gpurun_out/xp9
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_build.py --xp 1003,4200 --check 4200 --ref 1003 --rounds 2 > gpurun_out/xp9/chk.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,2256,2512,2768 --rounds 9 > gpurun_out/xp9/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,2256,2512 --rounds 5 > gpurun_out/xp9/sintel8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --dtype bf16 --B 8 --H 47 --W 156 --xp 100,2300,2301,2302 --rounds 7 > gpurun_out/xp9/kitti.log 2>&1 || exit $?
grep -h "xp\|bit" gpurun_out/xp9/*.log
