#!/bin/bash
# Nystrom bench under several group / lane / HW-queue configurations
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nys_tests.log 2>&1 || { tail -30 gpurun_out/nys_tests.log; exit 1; }
tail -1 gpurun_out/nys_tests.log
for cfg in $NYS_CFGS; do
  set -- $(echo $cfg | tr _ " ")
  OI_NYS_GROUPS=$1 OI_NYS_LANES=$2 GPU_MAX_HW_QUEUES=$3 timeout -k 10 200 python bench.py --workload nystrom --no-cpu-baseline --out gpurun_out/nyscfg.json > gpurun_out/nyscfg.log 2>&1 || { tail -20 gpurun_out/nyscfg.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/nyscfg.json'));print('groups',$1,'lanes',$2,'hwq',$3,'value',d['value'],'ms',d['ms_per_step'],'evals',d['evals_per_cell'],'evals/s',round(d['value']*d['evals_per_cell'],1))"
done
