set -u
O=gpurun_out/s3y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "variants and 50" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --workload sintel --variants 8,50 --rounds 7 > $O/ab.log 2>&1; echo "ab rc=$?"; tail -1 $O/ab.log
timeout -k 10 300 python -u scripts/ab_kernels.py --workload kitti --batch 8 --variants 8,50 --rounds 3 > $O/ab_k.log 2>&1; echo "ab rc=$?"; tail -1 $O/ab_k.log
