set -u
mkdir -p gpurun_out/xp3
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003,4048:16384,4050:16384,4051:16384,4052:16384,4048:20480,4048:24576,4048:28672 --rounds 7 > gpurun_out/xp3/sintel.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/xp_step.py --dtype bf16 --B 8 --H 47 --W 156 --xp 100,100:16384,2150:16384,2151:16384 --rounds 5 > gpurun_out/xp3/kitti.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_lookup.py --check 20480,24576,28672 --xp 0,16384,20480,24576,28672 --rounds 9 > gpurun_out/xp3/lookup.log 2>&1 || exit $?
grep -h xp gpurun_out/xp3/*.log
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,30 --check 30 > gpurun_out/xp3/alt.log 2>&1 || exit $?
grep -h xp gpurun_out/xp3/alt.log
