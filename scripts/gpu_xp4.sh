set -u
mkdir -p gpurun_out/xp4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/xp4/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/xp4/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/xp4/bench_sintel.json 2>gpurun_out/xp4/bench_sintel.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --workload kitti > gpurun_out/xp4/bench_kitti.json 2>gpurun_out/xp4/bench_kitti.err || exit $?
timeout -k 10 240 python -u scripts/xp_alt.py --xp 0,30 --rounds 7 > gpurun_out/xp4/alt.log 2>&1 || exit $?
python - <<'P'
import json
for f in ["sintel","kitti"]:
    d=json.load(open(f"gpurun_out/xp4/bench_{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["lookup_roofline"]["avg_launch_us"])
P
grep -h xp gpurun_out/xp4/alt.log
