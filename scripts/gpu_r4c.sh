#!/bin/bash
# Round-4 experiment session C: build store policy + timeline, lookup output
# stores through LDS, the bench with the round-4 product library.
set -u
O=gpurun_out/r4c
mkdir -p "$O"
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step build_store 200 python -u scripts/xp_build.py --shape 1x55x128 --xp 0 64 128 --split
step lookup_ts_sintel 200 python -u scripts/ab_step.py --workload sintel --variants -1 512 576 --reps 50 --rounds 7
step lookup_ts_b8 200 python -u scripts/ab_step.py --workload sintel --batch 8 --variants -1 512 --reps 10 --rounds 7
step lookup_ts_kitti 200 python -u scripts/ab_step.py --workload kitti --batch 8 --dtype bf16 --variants -1 512 --reps 10 --rounds 7
step bench_sintel 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline
step bench_driver 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
echo "== done"
