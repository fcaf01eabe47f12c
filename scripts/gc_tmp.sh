set -u
O=gpurun_out/s3w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $O/pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload chairs --steps 20 --warmup 3 --no-cpu-baseline > $O/chairs.log 2>&1; echo "chairs rc=$?"; tail -1 $O/chairs.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; l=d['lookup_roofline']; print(d['value'], r['kernel'][:30], r['achieved'], r['frac'], r['avg_launch_us'], l['avg_launch_us'])"
