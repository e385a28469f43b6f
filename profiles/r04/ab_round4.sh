#!/bin/bash
# Round-4 A/B session: -m gpu suite, then per-kernel A/B of the new k_blur_rows / k_describe_dma /
# batched-trial k_pose against the previous kernels (env switches), each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; tail -n 3 gpurun_out/pt.log
grep -E "^FAILED|^ERROR" gpurun_out/pt.log | head -20
# 0 = pass, 1 = test failures (keep measuring); anything else (crash, timeout, abort) ends the call
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/_kab.sh k_blur main COEB_BLUR_ROWS=0 main COEB_BLUR_ROWS=64 COEB_DESC_DMA=0 main COEB_DESC_DMA=4 main COEB_DESC_DMA=8 main || exit $?
bash tools/_kab.sh k_octree COEB_OCT_SPLIT=3 main COEB_OCT_SPLIT=5 main COEB_OCT_SPLIT=0 main || exit $?
bash tools/_dab.sh lib/var_tb1.so lib/var_tb2.so main || exit $?
# octree per-level clocks: config A batch and a config-B 32-frame shard
export COEB_SIDE_STREAM=0 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_octclk.so
timeout -k 10 120 python tools/_oct_timing.py > gpurun_out/oct_A.txt 2>&1 || { echo "oct_A rc=$?"; tail -5 gpurun_out/oct_A.txt; exit 1; }
cat gpurun_out/oct_A.txt
timeout -k 10 120 python tools/_oct_timing.py 1280 960 33 > gpurun_out/oct_B32.txt 2>&1 || { echo "oct_B rc=$?"; tail -5 gpurun_out/oct_B32.txt; exit 1; }
cat gpurun_out/oct_B32.txt
unset COEB_LIB_PATH COEB_SIDE_STREAM
# config B 64-frame shard (the 8-rank share of the 512-frame batch): level-0 octree at 1024 threads
for v in 0 64; do
  COEB_OCT_WIDE_F=$v COEB_OCT_SPLIT=0 timeout -k 10 200 python bench.py --config B --global-frames 64 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/b64_$v.log 2>&1 || { echo "b64 rc=$?"; tail -3 gpurun_out/b64_$v.log; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/b64_%s.log" % sys.argv[1]) if x.startswith("{")][-1])
k = d["kernels_ms_per_step"]
print("B64 wide=%s step=%.3f ms value=%.0f octree=%.3f match=%.3f" % (sys.argv[1], d["ms_per_step"], d["value"], k.get("k_octree", -1), k.get("k_match", -1)))
PY
done
