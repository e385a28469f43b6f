#!/bin/bash
# Vector-memory pipe counter passes (TA address / TD data / TCP L1) over config A, one 1025-frame
# pipeline, side stream off: are k_fast / k_describe bound by the L1 path rather than latency?
# Usage: tools/pipes_mem.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-pipes_mem}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp COEB_SIDE_STREAM=0
B="python bench.py --pipelines 1 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$out/$name" -o run -- $B \
        > "$out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc $*"
    [ $rc -ne 0 ] && { tail -n 5 "$out/$name.log"; exit $rc; }
    return 0
}
pass m1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
pass m2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUSY_avr GRBM_GUI_ACTIVE
pass m3 TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
pass m4 TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE
python tools/pmc_summary.py "$out"/m*/run_counter_collection.csv > "$out/summary.txt" 2>&1
grep -E "k_fast|k_describe|k_blur|k_pyr|k_octree|k_match" "$out/summary.txt"
