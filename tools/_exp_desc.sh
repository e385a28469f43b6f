#!/bin/bash
# k_describe keypoints-per-wave probe: parity at KP 4 / 16 (default 8 runs in gpu_session pytest),
# per-kernel A/B times, and FETCH_SIZE per launch at KP 4 / 8 / 32 (side stream off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/desc
export TMPDIR=/tmp
for kp in 4 16; do
  COEB_DESC_KP=$kp timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/desc/pytest_kp$kp.log 2>&1 \
    || { echo "pytest KP=$kp rc=$?"; tail -20 gpurun_out/desc/pytest_kp$kp.log; exit 1; }
  echo "pytest KP=$kp: $(tail -1 gpurun_out/desc/pytest_kp$kp.log)"
done
for kp in 4 8 32; do
  COEB_DESC_KP=$kp COEB_SIDE_STREAM=0 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/desc/f$kp -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras > gpurun_out/desc/f$kp.log 2>&1 || { echo "pmc KP=$kp rc=$?"; exit 1; }
  python tools/pmc_summary.py gpurun_out/desc/f$kp/run_counter_collection.csv --frames 257 > gpurun_out/desc/f$kp.txt 2>&1
  echo "KP=$kp $(grep k_describe gpurun_out/desc/f$kp.txt)"
done
