#!/bin/bash
# Round-4 A/B session 4: -m gpu suite (split matcher lists), k_fast at 8 workgroups per CU,
# config-B shards with / without split lists, octree single-wave upper levels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_kab.sh k_fast main lib/var_fast8p0.so main || exit $?
bash tools/_bab.sh 64 main COEB_MATCH_SPLIT=0 main COEB_MATCH_SPLIT=4 main COEB_MATCH_SPLIT=8 COEB_OCT_SPLIT=3 main COEB_OCT_SPLIT=1 main || exit $?
unset COEB_MATCH_SPLIT COEB_OCT_SPLIT
bash tools/_bab.sh 128 main COEB_MATCH_SPLIT=0 main || exit $?
unset COEB_MATCH_SPLIT
bash tools/_bab.sh 256 main COEB_MATCH_SPLIT=0 main COEB_MATCH_SPLIT=2 main || exit $?
unset COEB_MATCH_SPLIT
bash tools/_bab.sh 512 main || exit $?
bash tools/_kab.sh k_octree COEB_OCT_SPLIT=3 main COEB_OCT_SPLIT=5 main || exit $?
