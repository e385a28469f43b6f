#!/bin/bash
# round 5 session 5: default bench line (no CPU leg) + step timeline of the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/s5/bench.log 2>&1 || { tail -5 gpurun_out/s5/bench.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/s5/bench.log') if l.startswith('{')][-1]); print('value', d['value'], 'ms/step', d['ms_per_step'], d['kernels_ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s5/tl -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s5/tl.log 2>&1 || exit 1
python tools/timeline2.py gpurun_out/s5/tl/run_kernel_trace.csv 2 > gpurun_out/s5/timeline.txt 2>&1; tail -n 12 gpurun_out/s5/timeline.txt
