#!/bin/bash
# round 5 session 37: launch bounds for config A's kernels: k_describe at 6 waves per SIMD (80 VGPRs
# + 16 B scratch, var_desc6) and k_octree at 7 (72 VGPRs, 38 SGPR spills, var_oct7) against the
# build (88 / 78 VGPRs, 5 / 6 waves): parity, one-pipeline kernel times and the config-A step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s37
export TMPDIR=/tmp
for v in desc6 oct7; do
  COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "golden or extract_A or ragged or params or edge_images or B_" --timeout 120 --timeout-method thread > gpurun_out/s37/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/s37/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s37/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s37/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s37/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-8s step=%.4f ms value=%.0f describe=%.4f octree=%.4f' % ('$1', d['ms_per_step'], d['value'], k['k_describe'], k['k_octree']))"
}
for rep in 1 2 3; do
  run base main
  run desc6 desc6
  run oct7 oct7
done
