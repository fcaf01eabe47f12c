#!/bin/bash
# Round-3 re-entry check: smoke + full GPU suite, then quick bench lines per config.
set -u
bash scripts/gpu_tests.sh r03e || exit $?
bash scripts/gpu_quick.sh r03e_b "" "--workload sintel" "--workload sintel --layout nhwc" "--workload chairs" "--workload kitti" "--workload kitti --layout nhwc" "--workload sintel --batch 8" "--workload 1080p --block alt"
