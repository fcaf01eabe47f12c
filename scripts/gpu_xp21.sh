set -u
mkdir -p gpurun_out/xp21
export TMPDIR=/tmp
for H in 48 54 55 56 62 63; do
  timeout -k 10 120 python -u scripts/xp_build.py --H $H --xp 1003 --rounds 5 > gpurun_out/xp21/h$H.log 2>&1 || exit $?
  echo "H=$H $(grep '"xp"' gpurun_out/xp21/h$H.log)"
done
