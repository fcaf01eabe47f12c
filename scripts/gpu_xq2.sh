# On-the-fly kernel: product (f16 pair) vs NRB=2 vs the r01 3-way form; then the alt/config GPU tests.
set -o pipefail
O=gpurun_out/xq6.log
: > $O
timeout -k 10 200 python -u scripts/xp_alt.py --xp 0,8,9 >> $O 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_channels_last.py tests/test_e2e_flow.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $O 2>&1 || exit $?
