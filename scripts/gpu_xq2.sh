# Early-gather lookup (xp 200) vs the product lookup (0), bit-checked, three shapes.
set -o pipefail
O=gpurun_out/xq8.log
: > $O
timeout -k 10 120 python -u scripts/xp_lookup.py --xp 0,200,201 --check 200 >> $O 2>&1 || exit $?
timeout -k 10 120 python -u scripts/xp_lookup.py --B 8 --xp 0,200 --check 200 >> $O 2>&1 || exit $?
timeout -k 10 120 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp 0,200 --check 200 >> $O 2>&1 || exit $?
