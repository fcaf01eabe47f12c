set -u
mkdir -p gpurun_out/xp1
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_lookup.py --xp 0,4096,8192,12288,16384 --check 4096,8192,12288,16384 --rounds 9 > gpurun_out/xp1/b1.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --xp 0,4096,8192,12288,16384 --rounds 9 > gpurun_out/xp1/b8.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp 0,4096,12288 --check 4096,12288 --rounds 9 > gpurun_out/xp1/kitti.log 2>&1 || exit $?
cat gpurun_out/xp1/*.log | grep xp
