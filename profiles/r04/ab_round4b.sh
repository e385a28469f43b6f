#!/bin/bash
# Round-4 A/B session 2: -m gpu suite (batched-trial k_pose fix), k_fast old / scalar-strength /
# packed-strength, k_pose trial batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_kab.sh k_fast main lib/var_fastpk0.so lib/var_oldext.so main || exit $?
bash tools/_dab.sh lib/var_tb1.so lib/var_tb2.so main || exit $?
