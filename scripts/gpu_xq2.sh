# Fused lookup + convc1: r01 form (0) vs round-2 forms (1: 512 threads, 2: 1024), three shapes; then motion tests.
set -o pipefail
O=gpurun_out/xmo.log
: > $O
timeout -k 10 120 python -u scripts/xp_motion.py >> $O 2>&1 || exit $?
timeout -k 10 120 python -u scripts/xp_motion.py --B 2 >> $O 2>&1 || exit $?
timeout -k 10 150 python -u scripts/xp_motion.py --B 8 --H 47 --W 156 >> $O 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_motion.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $O 2>&1 || exit $?
