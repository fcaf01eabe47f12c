set -u
mkdir -p gpurun_out/xp5
export TMPDIR=/tmp
for sw in "30 3" "50 5" "300 50" "2000 200" "50 2000"; do
  set -- $sw
  timeout -k 10 300 python -u bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/xp5/b_$1_$2.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/xp5/b_$1_$2.json'));print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['lookup_roofline']['avg_launch_us'])"
done
timeout -k 10 300 python -u scripts/xp_step.py --xp 1003 --rounds 3 --steps 20 2>/dev/null | grep xp
