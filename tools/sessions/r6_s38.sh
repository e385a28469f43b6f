#!/bin/bash
# single-frame k_octree threads per workgroup (F == 1): 1024 (main) vs 256 (previous) vs 512
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s38; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_adapter_exec.py -q -x -m gpu \
    --timeout 120 --timeout-method thread -k "extract or golden or adapter" > $O/pt.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in main o256 o512; do
    if [ $v = main ]; then L=""; else L=coeb-slam_amd/lib/var_$v.so; fi
    COEB_LIB_PATH=$L timeout -k 10 120 python tools/single_frame.py 200 > $O/sf_${v}_$r.log 2>&1 || { tail -5 $O/sf_${v}_$r.log; exit 1; }
    echo "$v $r $(cat $O/sf_${v}_$r.log)"
  done
done
for v in main o256 o512; do
  if [ $v = main ]; then L=""; else L=coeb-slam_amd/lib/var_$v.so; fi
  COEB_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run -- python tools/single_frame.py 100 > $O/p_$v.log 2>&1 || { tail -5 $O/p_$v.log; exit 1; }
  f=$(find $O/p_$v -name '*kernel_stats.csv' | head -1); echo "$v: $(grep -h k_octree $f)"
done
