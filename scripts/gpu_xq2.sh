# Epilogue store-path experiments (split H2 and bf16 builds), bit-checked.
set -o pipefail
O=gpurun_out/xq3.log
: > $O
timeout -k 10 150 python -u scripts/xp_build.py --xp 1003,2096,2064 --ref 1003 --check 2096,2064 >> $O 2>&1 || exit $?
timeout -k 10 150 python -u scripts/xp_build.py --dtype bf16 --B 8 --H 47 --W 156 --xp 0,164,196,100,264 --ref 0 --check 164,196,264 >> $O 2>&1 || exit $?
timeout -k 10 150 python -u scripts/xp_step.py --xp 1003,2032,2064,2096 >> $O 2>&1 || exit $?
