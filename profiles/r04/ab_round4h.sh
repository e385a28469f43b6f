#!/bin/bash
# Round-4 A/B session 8: the pending changes (packed-arc FAST strength, per-wave LM state in
# k_pose, small-batch octree key capacity) built as lib/var_pend.so: the -m gpu suite on it, then
# each change against the in-tree library (lib/var_noarc.so = var_pend without the packed arc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_pend.so timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_kab.sh k_fast main lib/var_pend.so lib/var_noarc.so main lib/var_pend.so || exit $?
bash tools/_dab.sh main lib/var_pend.so main lib/var_pend.so || exit $?
export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_pend.so
timeout -k 10 200 python tools/_pose_timing.py || exit $?
unset COEB_LIB_PATH
bash tools/_bab.sh 64 main lib/var_pend.so COEB_OCT_KL_SMALL=0 lib/var_pend.so || exit $?
unset COEB_OCT_KL_SMALL
bash tools/_bab.sh 512 main lib/var_pend.so || exit $?
