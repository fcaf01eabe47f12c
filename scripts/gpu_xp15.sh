set -u
mkdir -p gpurun_out/xp15
export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/xp15/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/xp15/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xp15/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/xp15/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload 1080p --block alt --no-cpu-baseline > gpurun_out/xp15/alt.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/xp15/alt.json'));print(d['value'], d['roofline']['avg_launch_us'])"
