set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcA gpurun_out/pmcB
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcA -o run --output-format csv -- python scripts/pmc_panel.py > gpurun_out/pmcA.log 2>&1 || { tail -20 gpurun_out/pmcA.log; exit 1; }
python scripts/pmc_kernels.py gpurun_out/pmcA
