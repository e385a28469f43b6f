#!/bin/bash
# round 6 session 9: full GPU suite on the current build, D and A lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/s9; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; }
grep -E "\{'frames'" $O/pytest_gpu.log | cut -c1-200
for c in D D A; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > $O/bench$c.log 2>&1 || { tail -5 $O/bench$c.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$O/bench$c.log') if l.startswith('{')][-1]); print('$c', d['value'], d['ms_per_step'], d['parity_sample']['bit_exact'] if 'parity_sample' in d else None)"
done
