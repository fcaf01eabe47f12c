set -u
O=gpurun_out/s3f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/ab_lookup.py --variants 0,1,94,95,96,97,91,93 > $O/ab_lookup.log 2>&1; echo "abl rc=$?"; tail -1 $O/ab_lookup.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python -u scripts/ab_lookup.py --variants 0,94 --rounds 2 > $O/prof.log 2>&1; echo "prof rc=$?"
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name '*kernel_trace.csv' -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/prof
