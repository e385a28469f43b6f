#!/bin/bash
# k_describe L2 reuse probe: FETCH_SIZE per frame at batch 16, 64, 256 (side stream
# off so every kernel is one batch launch), then the k_fast phase clocks (COEB_FAST_CLOCK build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/l2
export COEB_SIDE_STREAM=0 TMPDIR=/tmp
for b in 16 64 256; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/l2/b$b -o run -- \
    python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras > gpurun_out/l2/b$b.log 2>&1 || { echo "pmc b$b rc=$?"; exit 1; }
  python tools/pmc_summary.py gpurun_out/l2/b$b/run_counter_collection.csv --frames $((b + 1)) > gpurun_out/l2/b$b.txt 2>&1
  echo "== batch $b"; grep -E "k_describe|k_blur|k_fast" gpurun_out/l2/b$b.txt
done
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_fastclk.so timeout -k 10 120 python tools/_fast_timing.py > gpurun_out/l2/fastclk.log 2>&1 || { echo "fastclk rc=$?"; exit 1; }
cat gpurun_out/l2/fastclk.log
