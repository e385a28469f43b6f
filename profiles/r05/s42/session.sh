#!/bin/bash
# round 5 session 42: cornerSubPix LDS row paddings (term rows NL + 5 doubles, at least that: the sink slot; trp1 failed parity, patch rows BW + 1
# floats in the build; 2.7 bank-conflict cycles per LDS instruction in pmcD): parity, k_subpix alone
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s42
export TMPDIR=/tmp
for v in trp7 trp9 prp3 prp5; do
  COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_flow.py -q -x -m gpu -k "subpix or process_moving" --timeout 120 --timeout-method thread > gpurun_out/s42/pt_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 gpurun_out/s42/pt_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
run() {   # tag lib
  if [ $2 = main ]; then unset COEB_LIB_PATH; else export COEB_LIB_PATH=$PWD/coeb-slam_amd/lib/var_$2.so; fi
  timeout -k 10 240 python bench.py --config D --steps 6 --warmup 2 --no-cpu-baseline --no-extras --no-e2e > gpurun_out/s42/$1.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/s42/$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s42/$1.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print('%-6s step=%.4f ms value=%.0f k_subpix=%.4f' % ('$1', d['ms_per_step'], d['value'], k['k_subpix']))"
}
for rep in 1 2; do
  run base main
  for v in trp7 trp9 prp3 prp5; do run $v $v; done
done
