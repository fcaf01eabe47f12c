#!/bin/bash
# Round-4 experiment session A (via gpurun, repo root): persistent / staggered /
# late-DMA f32 builds, the level-by-XCD on-the-fly lookup, and the new bench
# build timing.  Every GPU step has its own time limit; the first failure ends it.
set -u
O=gpurun_out/r4a
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -n 4 "$O/$n.log"
  [ $rc -eq 0 ] || exit $rc
}
step bench_driver1 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
step diag_gap 400 python -u scripts/diag_driver_gap.py --rounds 3
step bench_driver2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
step persist_sintel 240 python -u scripts/xp_persist.py --shape 1x55x128
step alt_xl 240 python -u scripts/ab_step.py --workload 1080p --block alt --variants -2 106 107 --reps 5 --rounds 5
step bench_sintel 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline
step persist_b8 240 python -u scripts/xp_persist.py --shape 8x55x128 --variants prod prodL p512 p512L p512s1000 --trace ""
step strip_kitti 240 python -u scripts/xp_strip.py --shape 8x47x156 --dtype bf16 --strips 8 16 30 60
step strip_sintel 240 python -u scripts/xp_strip.py --shape 1x55x128 --strips 8 16 28 56
echo "== done"
