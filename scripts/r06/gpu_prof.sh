#!/bin/bash
# round 6 profiles of the driver's bench command (GPU leg): GPU tests, kernel
# trace + stats, then PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters), each its
# own run; summaries to gpurun_out/prof_$TAG/ (copied to profiles/r06 by hand)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r06}
D=gpurun_out/prof_$TAG
mkdir -p $D
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "not fit_large" > $D/gputests.log 2>&1
  rc=$?; tail -2 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
fi
CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/trace -o run --output-format csv -- $CMD > $D/bench_under_rocprof.json 2> $D/trace.err
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/trace.err; exit $rc; }
python3 scripts/trace_summary.py $D/trace > $D/trace_summary.txt
find $D/trace -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
find $D/trace -name "*kernel_trace.csv" -delete
timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $D/pmcF -o run --output-format csv -- $CMD > $D/pmcF.json 2> $D/pmcF.err
rc=$?; echo "fetch rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/pmcF.err; exit $rc; }
timeout -s KILL 420 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $D/pmcW -o run --output-format csv -- $CMD > $D/pmcW.json 2> $D/pmcW.err
rc=$?; echo "write rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/pmcW.err; exit $rc; }
python3 scripts/pmc_summary.py $D/pmcF $D/pmcW > $D/pmc_hbm_summary.json
rm -rf $D/pmcF $D/pmcW
timeout -s KILL 420 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $D/pmcS -o run --output-format csv -- $CMD > $D/pmcS.json 2> $D/pmcS.err
rc=$?; echo "sq rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/pmcS.err; exit $rc; }
python3 scripts/pmc_kernels.py $D/pmcS > $D/pmc_sq.txt
rm -rf $D/pmcS
du -sh $D; head -c 600 $D/kernel_stats.csv; echo; cut -c1-200 $D/pmc_sq.txt | head -8
