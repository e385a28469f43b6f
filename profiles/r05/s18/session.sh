#!/bin/bash
# round 5 session 18: k_pyr_rows workgroups 512 columns wide (default) vs stacked 128 x 32: parity,
# kernel A/B, FETCH_SIZE of both, config A step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "blur_pyramid or golden_extract or extract_A or extract_B or ragged or params or edge_images" --timeout 120 --timeout-method thread > gpurun_out/s18/pt.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/s18/pt.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/_kab.sh k_pyr_level main lib/var_pyrstack.so main lib/var_pyrstack.so || exit 1
B="python bench.py --pipelines 1 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
for v in main pyrstack; do
  if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
  COEB_SIDE_STREAM=0 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/s18/f_$v -o run -- $B > gpurun_out/s18/f_$v.log 2>&1 || exit 1
done
unset COEB_LIB_PATH
python - <<'PY'
import csv
for v in ("main", "pyrstack"):
    t = [float(r["Counter_Value"]) for r in csv.DictReader(open("gpurun_out/s18/f_%s/run_counter_collection.csv" % v)) if "k_pyr_rows" in r["Kernel_Name"]]
    print(v, "pyramid FETCH_SIZE x2 per pyramid: %.0f MB" % (2 * sum(t) * 1024 / 1e6 / (len(t) / 7)))
PY
for rep in 1 2; do
  for v in main pyrstack; do
    if [ $v = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so; fi
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s18/step_$v.log 2>&1 || exit 1
    python -c "import json; d=json.loads([l for l in open('gpurun_out/s18/step_$v.log') if l.startswith('{')][-1]); print('%-10s step=%.4f ms value=%.0f' % ('$v', d['ms_per_step'], d['value']))"
  done
done
