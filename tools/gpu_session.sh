#!/bin/bash
# One gpurun session: each GPU step has its own time limit; stop at the first fault/timeout
# (exit codes other than 0 = pass and 1 = test failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 to=$2
    shift 2
    local t0=$(date +%s)
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
    tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for step in "$@"; do
    case "$step" in
        pytest) run pytest_gpu 900 python -m pytest tests -q -m gpu -x ;;
        pytestall) run pytest_gpu 900 python -m pytest tests -q -m gpu ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        benchB) run benchB 600 python bench.py --config B --batch 64 --no-cpu-baseline ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --no-cpu-baseline ;;
        diag) run diag 600 python tools/diag_parity.py ;;
        *) echo "unknown step $step" ;;
    esac
done
