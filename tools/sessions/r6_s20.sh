#!/bin/bash
# round 6 session 20: k_match phase clocks (A: 1025 pairs; B shard: 33) and k_fast per-cell phase clocks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s20; mkdir -p $O; export TMPDIR=/tmp
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_mclock.so timeout -k 10 300 python tools/_match_timing.py 640 480 1025 1000 > $O/match_timing_A.txt 2>&1 || { tail -5 $O/match_timing_A.txt; exit 1; }
cat $O/match_timing_A.txt
COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_mclock.so timeout -k 10 300 python tools/_match_timing.py 640 480 257 1000 > $O/match_timing_A257.txt 2>&1 || { tail -5 $O/match_timing_A257.txt; exit 1; }
cat $O/match_timing_A257.txt
COEB_SIDE_STREAM=0 COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_fclock.so timeout -k 10 300 python tools/_fast_timing.py > $O/fast_timing.txt 2>&1 || { tail -5 $O/fast_timing.txt; exit 1; }
cat $O/fast_timing.txt
