set -u
mkdir -p gpurun_out/xp10
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_motion.py --xp 1,2,3,4 > gpurun_out/xp10/m1.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_motion.py --B 2 --xp 1,3 > gpurun_out/xp10/m2.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_motion.py --B 8 --H 47 --W 156 --xp 1,3 > gpurun_out/xp10/m8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,1013 --rounds 9 > gpurun_out/xp10/remap1.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,1013 --rounds 5 > gpurun_out/xp10/remap8.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp10/*.log
