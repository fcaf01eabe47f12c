set -u
mkdir -p gpurun_out/xp12
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,40,43,44,45,46,47,48 --rounds 7 > gpurun_out/xp12/iid.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,43,44,47,48 --rounds 7 --smooth 16 > gpurun_out/xp12/smooth.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp12/*.log
