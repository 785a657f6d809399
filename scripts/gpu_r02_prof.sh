#!/bin/bash
# round 2 profiles of the driver's bench command: kernel trace + stats, then PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ busy/conflict counters), each pass its own run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r02}
CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
mkdir -p gpurun_out/prof_$TAG gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG gpurun_out/pmcS_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $CMD > gpurun_out/bench_${TAG}_under_rocprof.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.err; exit $rc; }
timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcF_$TAG -o run --output-format csv -- $CMD > gpurun_out/pmcF_$TAG.json 2> gpurun_out/pmcF_$TAG.err
rc=$?; echo "fetch rc $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcF_$TAG.err; exit $rc; }
timeout -s KILL 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcW_$TAG -o run --output-format csv -- $CMD > gpurun_out/pmcW_$TAG.json 2> gpurun_out/pmcW_$TAG.err
rc=$?; echo "write rc $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcW_$TAG.err; exit $rc; }
python3 scripts/pmc_summary.py gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG > gpurun_out/pmc_summary_$TAG.json
rm -rf gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG   # raw per-dispatch csv: hundreds of MB
timeout -s KILL 420 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcS_$TAG -o run --output-format csv -- $CMD > gpurun_out/pmcS_$TAG.json 2> gpurun_out/pmcS_$TAG.err
rc=$?; echo "sq rc $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcS_$TAG.err; exit $rc; }
python3 scripts/pmc_kernels.py gpurun_out/pmcS_$TAG > gpurun_out/pmc_sq_$TAG.txt
rm -rf gpurun_out/pmcS_$TAG
# keep the stats and a trace summary, not the 170k-row trace
python3 scripts/trace_summary.py gpurun_out/prof_$TAG > gpurun_out/trace_summary_$TAG.txt
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
du -sh gpurun_out
echo done
