set -u
mkdir -p gpurun_out/s3b
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_bias.py sintel 0,10 > gpurun_out/s3b/diag.log 2>&1; echo "diag rc=$?"; tail -1 gpurun_out/s3b/diag.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s3b/pytest.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/s3b/pytest.log
timeout -k 10 300 python -u scripts/ab_kernels.py --workload sintel --variants 0,10 --rounds 5 > gpurun_out/s3b/ab.log 2>&1; echo "ab rc=$?"; tail -8 gpurun_out/s3b/ab.log
