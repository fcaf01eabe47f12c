set -u
mkdir -p gpurun_out/xp17
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_lookup.py --xp 0,201,202,203 --check 201,202,203 --rounds 9 > gpurun_out/xp17/b1.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --xp 0,202,203,204,206 --check 203 --rounds 9 > gpurun_out/xp17/b8.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp 0,202,203,204 --check 203 --rounds 9 > gpurun_out/xp17/kitti.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp17/*.log
