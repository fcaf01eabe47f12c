# GPU tests + Sintel and KITTI bench lines after adopting the r02 build changes.
set -u
OUT=gpurun_out/r2b
mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 $OUT/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_sintel 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline
run bench_kitti 200 python -u bench.py --workload kitti --steps 10 --warmup 2 --no-cpu-baseline
