set -u
export TMPDIR=/tmp
bash scripts/gpu_profile.sh xp8/sintel sintel_b1_f32 || exit $?
cat gpurun_out/xp8/sintel/trace_gaps.json
python - <<'P'
import json,csv
d=json.load(open("gpurun_out/xp8/sintel/bench_under_rocprof.json"))
print("under rocprof:", d["value"], d["roofline"]["avg_launch_us"], d["lookup_roofline"]["avg_launch_us"])
d=json.loads(open("gpurun_out/xp8/sintel/bench.log").read().strip().splitlines()[-1])
print("bench:", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"], d["lookup_roofline"]["avg_launch_us"])
for r in csv.DictReader(open("gpurun_out/xp8/sintel/kernel_stats.csv")):
    if "corr_" in r["Name"]: print(r["Name"][:60], r["Calls"], r["AverageNs"])
P
