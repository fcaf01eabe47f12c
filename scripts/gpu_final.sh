#!/bin/bash
# Round-end GPU session (via gpurun, repo root).  Parts, in order (default all):
#   tests    smoke + the whole -m gpu suite (scripts/gpu_tests.sh)
#   profiles bench line + rocprofv3 kernel stats + trace timeline + FETCH/WRITE
#            passes per BASELINE config (scripts/gpu_profile.sh)
#   backward training-step timing and peak memory (scripts/time_backward.py)
#   driver   the round driver's own bench command
# Outputs under gpurun_out/<round>/.  The first failing part ends the session.
# Usage: bash scripts/gpu_final.sh <round, e.g. r05> [part ...]
set -u
R=${1:-r05}
shift || true
PARTS=${*:-tests profiles backward driver}
export TMPDIR=/tmp
for P in $PARTS; do
  case $P in
    tests) bash scripts/gpu_tests.sh $R || exit $? ;;
    profiles)
      bash scripts/gpu_profile.sh $R/sintel sintel_b1_f32 || exit $?
      bash scripts/gpu_profile.sh $R/chairs chairs_b1_f32 --workload chairs || exit $?
      bash scripts/gpu_profile.sh $R/kitti kitti_b8_bf16 --workload kitti || exit $?
      bash scripts/gpu_profile.sh $R/kitti_nhwc kitti_b8_bf16 --workload kitti --layout nhwc || exit $?
      bash scripts/gpu_profile.sh $R/sintel_b8 sintel_b8_f32 --batch 8 || exit $?
      bash scripts/gpu_profile.sh $R/hd_alt 1080p_b1_f32 --workload 1080p --block alt || exit $?
      bash scripts/gpu_profile.sh $R/hd_full 1080p_b1_f32 --workload 1080p || exit $? ;;
    backward)
      mkdir -p gpurun_out/$R/backward
      for W in sintel chairs; do
        timeout -k 10 200 python -u scripts/time_backward.py --workload $W \
          > gpurun_out/$R/backward/time_backward_$W.log 2>&1 || exit $?
      done ;;
    driver)
      mkdir -p gpurun_out/$R
      timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
        > gpurun_out/$R/bench_driver_cmd.log 2>&1 || exit $? ;;
    *) echo "unknown part $P"; exit 2 ;;
  esac
  echo "== $P done"
done
