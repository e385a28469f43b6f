#!/bin/bash
# Kernel timeline of the default bench with the side stream on (as the bench line runs it):
# rocprofv3 kernel trace of 3 steps, then tools/timeline.py prints each launch's start / end
# relative to the step start and the busy time per stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tl2
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl2/t -o run -- \
  python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-profile --no-e2e --no-extras > gpurun_out/tl2/b.log 2>&1 || { echo "trace rc=$?"; exit 1; }
python tools/timeline.py gpurun_out/tl2/t/run_kernel_trace.csv > gpurun_out/tl2/timeline.txt 2>&1; tail -40 gpurun_out/tl2/timeline.txt
