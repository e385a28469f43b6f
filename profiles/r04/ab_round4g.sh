#!/bin/bash
# Round-4 A/B session 7: -m gpu suite (one wave per batched k_pose trial), first-round trial
# count, k_blur_rows band height.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_dab.sh main lib/var_t1_2.so lib/var_t1_4.so main || exit $?
timeout -k 10 200 python tools/_pose_timing.py || exit $?
bash tools/_kab.sh k_blur COEB_BLUR_ROWS=16 main COEB_BLUR_ROWS=24 main COEB_BLUR_ROWS=32 main || exit $?
