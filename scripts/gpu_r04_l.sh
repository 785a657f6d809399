# round 4: kernel trace of the eigensolver probe
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r04/eigh_trace; mkdir -p $D
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- tools/eigh_probe 928 32 > $D/probe.txt 2>&1 || { tail -20 $D/probe.txt; exit 1; }
find $D/t -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
find $D/t -name "*kernel_trace.csv" -exec cp {} $D/kernel_trace.csv \;
rm -rf $D/t
head -20 $D/kernel_stats.csv
