set -u
mkdir -p gpurun_out/xp11
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,40,41 --rounds 7 > gpurun_out/xp11/iid.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,40,41 --rounds 7 --smooth 16 > gpurun_out/xp11/smooth.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,40 --rounds 5 --H 55 --W 128 > gpurun_out/xp11/sintel.log 2>&1 || exit $?
grep -h "xp" gpurun_out/xp11/*.log
