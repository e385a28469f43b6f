#!/bin/bash
# single-frame drop-in path: parity of the host-buffer entry points, timing (Python and C++),
# kernel / copy trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_adapter_exec.py tests/test_gpu_flow.py -q -x -m gpu \
    --timeout 120 --timeout-method thread -k "extract or stereo or match or golden or adapter or localmap or keyframe or pose" > $O/pt.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pt.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 180 python tools/single_frame.py > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
cat $O/plain.log
timeout -k 10 120 python -c "import sys; sys.path.insert(0, 'coeb-slam_amd'); import bench, json; print(json.dumps(bench.single_frame_cpp(640, 480)))" > $O/cpp.log 2>&1 || { tail -5 $O/cpp.log; exit 1; }
cat $O/cpp.log
COEB_SIDE_STREAM=0 timeout -k 10 120 python -c "import sys; sys.path.insert(0, 'coeb-slam_amd'); import bench, json; print(json.dumps(bench.single_frame_cpp(640, 480)))" > $O/cpp_noside.log 2>&1 || { tail -5 $O/cpp_noside.log; exit 1; }
echo "no side stream:"; cat $O/cpp_noside.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python tools/single_frame.py > $O/traced.log 2>&1 || { tail -5 $O/traced.log; exit 1; }
python tools/sf_timeline.py $O/tr > $O/breakdown.txt 2>&1; tail -40 $O/breakdown.txt
