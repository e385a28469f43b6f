#!/bin/bash
# round 6 session 24: k_octree per-workgroup clocks (config A, 257 and 512 frames)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s24; mkdir -p $O; export TMPDIR=/tmp
for F in 257 512; do
  COEB_SIDE_STREAM=0 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_oclock.so timeout -k 10 300 python tools/_oct_timing.py 640 480 $F > $O/oct_timing_$F.txt 2>&1 || { tail -5 $O/oct_timing_$F.txt; exit 1; }
  echo "== F=$F"; cat $O/oct_timing_$F.txt
done
