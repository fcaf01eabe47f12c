# On-the-fly kernel with pre-split operands (-1) vs the product's in-kernel split (-2) and the exp kernel (0); tests.
set -o pipefail
O=gpurun_out/xq7.log
: > $O
timeout -k 10 200 python -u scripts/xp_alt.py --xp 0,-1,-2 >> $O 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_channels_last.py tests/test_e2e_flow.py tests/test_gpu_graph.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $O 2>&1 || exit $?
