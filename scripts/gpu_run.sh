#!/bin/bash
# Generic GPU session (via gpurun, repo root): run each quoted command in turn
# under its own time limit, output to gpurun_out/<tag>/<i>.log; stop at the
# first command that fails (no retries).  Used for same-process A/Bs
# (scripts/ab_step.py, ab_build.py, ...) so that no one-off session file is
# needed: the gpurun command line is the record.
# Usage: bash scripts/gpu_run.sh <tag> <seconds per command> "<cmd 1>" ["<cmd 2>" ...]
set -u
TAG=$1; SECS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  echo "== [$i] $C" | tee -a "$OUT/commands.txt"
  timeout -k 10 "$SECS" bash -c "$C" > "$OUT/$i.log" 2>&1
  rc=$?
  echo "== [$i] rc=$rc"
  tail -n 4 "$OUT/$i.log"
  [ $rc -eq 0 ] || exit $rc
done
echo "== done"
