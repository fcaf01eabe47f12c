set -u
O=gpurun_out/s3u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "alt or Alternate" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|EPE" $O/pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
DXR_ALT_VARIANT=0 timeout -k 10 300 python -u bench.py --workload 1080p --block alt --steps 5 --warmup 1 --no-cpu-baseline > $O/hd_0.log 2>&1; echo "v0 rc=$?"; tail -1 $O/hd_0.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['achieved'], r['frac'], r['avg_launch_us'])"
