#!/bin/bash
# One SQ counter pass over the default bench (side stream off): issue stalls split into LDS and
# other, LDS bank-conflict cycles vs LDS-array cycles, per kernel.  Usage: tools/_exp_sq.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-sq}
mkdir -p gpurun_out/$tag
export COEB_SIDE_STREAM=0 TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_ANY \
  --kernel-trace --output-format csv -d gpurun_out/$tag/p -o run -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras > gpurun_out/$tag/p.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
python tools/pmc_summary.py gpurun_out/$tag/p/run_counter_collection.csv --frames 257 > gpurun_out/$tag/p.txt 2>&1
grep -E "k_fast|k_describe|k_blur|k_pyr|k_octree|k_match" gpurun_out/$tag/p.txt
