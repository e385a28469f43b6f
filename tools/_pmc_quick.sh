#!/bin/bash
# Two SQ counter passes of a short bench run, summarised per kernel: tools/_pmc_quick.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp COEB_SIDE_STREAM=0
tag=$1
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc_${tag}_a -o run -- $B > gpurun_out/pmc_${tag}_a.log 2>&1 || { echo "pass a failed"; tail -5 gpurun_out/pmc_${tag}_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_${tag}_b -o run -- $B > gpurun_out/pmc_${tag}_b.log 2>&1 || { echo "pass b failed"; tail -5 gpurun_out/pmc_${tag}_b.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_${tag}_a/run_counter_collection.csv gpurun_out/pmc_${tag}_b/run_counter_collection.csv --valu-json gpurun_out/pmc_${tag}_valu.json --frames 257 --command "$B" | grep -E "k_fast|k_describe|k_blur|k_pyr" 
