set -u
O=gpurun_out/s3q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "backward or e2e" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|max\|err|EPE" $O/pytest.log | tail -30
