#!/bin/bash
# Kernel timeline of one config-B step at FRAMES global frames (two pipelines): tools/_tl_b.sh FRAMES
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
g=${1:-64}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlb$g -o run -- python bench.py --config B --global-frames $g --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/tlb$g.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/tlb$g.log; exit 1; }
python tools/timeline2.py gpurun_out/tlb$g/run_kernel_trace.csv 2 > gpurun_out/timeline_b$g.txt 2>&1; cat gpurun_out/timeline_b$g.txt
