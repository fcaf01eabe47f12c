# Full-step A/B: bf16 KITTI B=8 build variants (q2 with / without non-temporal stores, one-block kernel).
set -o pipefail
O=gpurun_out/xq4.log
: > $O
timeout -k 10 200 python -u scripts/xp_step.py --dtype bf16 --B 8 --H 47 --W 156 --steps 5 --xp 0,100,264 >> $O 2>&1 || exit $?
timeout -k 10 150 python -u scripts/xp_step.py --xp 1003,2032,2064 >> $O 2>&1 || exit $?
