set -u
mkdir -p gpurun_out/xp2
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,1003:16384,4048,4048:16384,2064:16384 --rounds 7 > gpurun_out/xp2/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --B 8 --xp 1003,1003:16384,4048:16384 --rounds 5 > gpurun_out/xp2/sintel_b8.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --dtype bf16 --B 8 --H 47 --W 156 --xp 100,100:16384,2148,2148:16384 --rounds 5 > gpurun_out/xp2/kitti.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp 0,16384 --check 16384 --rounds 9 > gpurun_out/xp2/kitti_lookup.log 2>&1 || exit $?
grep -h xp gpurun_out/xp2/*.log
