#!/bin/bash
# config-1 latency: probe with/without per-launch events, then a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-single}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 200 python3 scripts/single_latency.py 200 8 > gpurun_out/single_$TAG.json 2> gpurun_out/single_$TAG.err
rc=$?; echo "probe rc $rc"; cat gpurun_out/single_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/single_$TAG.err; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 scripts/single_latency.py 200 4 > /dev/null 2> gpurun_out/prof_$TAG.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.err; exit $rc; }
python3 scripts/trace_summary.py gpurun_out/prof_$TAG > gpurun_out/trace_summary_$TAG.txt
python3 scripts/trace_rounds.py gpurun_out/prof_$TAG > gpurun_out/trace_rounds_$TAG.txt
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
