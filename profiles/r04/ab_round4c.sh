#!/bin/bash
# Round-4 A/B session 3: -m gpu suite (team-partition octree, fenced global keys, smaller k_fast
# lists), k_fast scalar vs packed strength, octree old vs new on configs A and B shards,
# octree per-level clocks of a config-B 33-frame batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_kab.sh k_octree main lib/var_fastlds_pk0.so lib/var_fast8p0.so lib/var_fast8.so lib/var_octold.so main || exit $?
bash tools/_bab.sh 64 main lib/var_octold.so COEB_OCT_KL=4096 main COEB_OCT_WIDE_F=64 main || exit $?
unset COEB_OCT_KL COEB_OCT_WIDE_F
bash tools/_bab.sh 512 main lib/var_octold.so || exit $?
export COEB_SIDE_STREAM=0 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_octclk2.so
timeout -k 10 120 python tools/_oct_timing.py 1280 960 33 > gpurun_out/oct_B32.txt 2>&1 || { echo "oct_B rc=$?"; tail -5 gpurun_out/oct_B32.txt; exit 1; }
cat gpurun_out/oct_B32.txt
timeout -k 10 120 python tools/_oct_timing.py > gpurun_out/oct_A.txt 2>&1 || { echo "oct_A rc=$?"; tail -5 gpurun_out/oct_A.txt; exit 1; }
cat gpurun_out/oct_A.txt
