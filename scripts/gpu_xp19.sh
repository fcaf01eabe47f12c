set -u
mkdir -p gpurun_out/xp19
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,60 --rounds 9 > gpurun_out/xp19/iid.log 2>&1 || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,60 --rounds 9 --smooth 16 > gpurun_out/xp19/smooth.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "alt or Alt or alternate or Alternate" > gpurun_out/xp19/pytest_alt.log 2>&1; rc=$?; tail -2 gpurun_out/xp19/pytest_alt.log; [ $rc -eq 0 ] || exit $rc
grep -h "xp" gpurun_out/xp19/*.log
