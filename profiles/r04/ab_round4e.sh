#!/bin/bash
# Round-4 A/B session 5: -m gpu suite (split k_match at small LDS), config-B shard variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_bab.sh 64 main COEB_MATCH_SPLIT_FULL=1 main COEB_MATCH_SPLIT_FULL=0 COEB_MATCH_LISTS_LDS=0 main COEB_MATCH_LISTS_LDS=1 COEB_OCT_KL=4096 main COEB_OCT_KL=2048 main || exit $?
unset COEB_MATCH_SPLIT_FULL COEB_MATCH_LISTS_LDS COEB_OCT_KL
bash tools/_bab.sh 512 main || exit $?
bash tools/_tl_b.sh 64 || exit $?
