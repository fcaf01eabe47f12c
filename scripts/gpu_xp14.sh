set -u
mkdir -p gpurun_out/xp14
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,41,50,51,52,53,54 --rounds 5 > gpurun_out/xp14/iid.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,50 --rounds 5 --smooth 16 > gpurun_out/xp14/smooth16.log 2>&1 || exit $?
grep -h "xp\|bin_dec" gpurun_out/xp14/*.log
