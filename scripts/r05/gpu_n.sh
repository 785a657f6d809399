# round 5: kernel stats of the eigensolver probe (64 matrices, M = 928) with
# 128-column orthogonalisation blocks (default)
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r05/${TAG:-n}; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- tools/eigh_probe 928 64 > $D/probe.txt 2> $D/trace.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/trace.err; exit $rc; }
find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
rm -rf $D/trace
cut -c1-160 $D/kernel_stats.csv | head -24
