set -u
mkdir -p gpurun_out/xp7
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_build.py --xp 1003,4200 --check 4200 --ref 1003 --rounds 3 > gpurun_out/xp7/chk_f32.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_build.py --dtype bf16 --B 8 --H 47 --W 156 --xp 100,2200,2201 --check 2200,2201 --ref 100 --rounds 3 > gpurun_out/xp7/chk_bf16.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,4200 --rounds 9 > gpurun_out/xp7/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,4200 --rounds 5 > gpurun_out/xp7/sintel8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --dtype bf16 --B 8 --H 47 --W 156 --xp 100,2200,2201 --rounds 7 > gpurun_out/xp7/kitti.log 2>&1 || exit $?
grep -h "xp\|bit" gpurun_out/xp7/*.log
