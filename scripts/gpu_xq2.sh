# Lookup tap-span staging A/B (xp 0 = product, xp 8 = full 11x16 staging), bit-checked; then parity.
set -o pipefail
O=gpurun_out/xq5.log
: > $O
timeout -k 10 120 python -u scripts/xp_lookup.py --xp 0,8 --check 8 >> $O 2>&1 || exit $?
timeout -k 10 120 python -u scripts/xp_lookup.py --B 8 --xp 0,8 --check 8 >> $O 2>&1 || exit $?
timeout -k 10 120 python -u scripts/xp_lookup.py --B 8 --H 47 --W 156 --dtype bf16 --xp 0,8 --check 8 >> $O 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $O 2>&1 || exit $?
