set -u
O=gpurun_out/s3l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"; tail -3 $O/bench.log
