set -u
mkdir -p gpurun_out/xp13
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,44,50 --rounds 7 > gpurun_out/xp13/iid.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,50 --rounds 7 --smooth 16 > gpurun_out/xp13/smooth16.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,50 --rounds 7 --smooth 64 > gpurun_out/xp13/smooth64.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,50 --rounds 5 --H 55 --W 128 > gpurun_out/xp13/sintel.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp13/*.log
