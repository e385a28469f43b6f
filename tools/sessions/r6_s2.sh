#!/bin/bash
# round 6 session 2: full GPU suite on the cleaned-up build, k_match kernarg A/B, config D line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; }
bash tools/_kab.sh k_match main lib/var_r6base.so main lib/var_r6base.so > $O/kab_match.log 2>&1; cat $O/kab_match.log
timeout -k 10 300 python bench.py --config D --no-cpu-baseline --no-extras > $O/benchD.log 2>&1 || { tail -5 $O/benchD.log; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/benchD.log') if l.startswith('{')][-1]); print('D', d['value'], d['ms_per_step'], d['kernels_ms_per_step'])"
