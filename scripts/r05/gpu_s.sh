# round 5: kernel stats of the Nystrom line (3 steps)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r05/${TAG:-s}; mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- python3 bench.py --workload nystrom --steps 3 --warmup 1 --no-cpu-baseline --out $D/nystrom.json > $D/nys_prof.log 2> $D/trace.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/trace.err; exit $rc; }
find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
rm -rf $D/trace
cut -c1-140 $D/kernel_stats.csv | head -30
