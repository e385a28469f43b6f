#!/bin/bash
# Per-pipe SQ counter passes over config A (one 1025-frame pipeline, side stream off, so each
# kernel is one whole-batch launch running alone): where do k_fast / k_describe / k_blur waves
# spend their cycles?  Counters missing from this rocprofv3's list are dropped, and every pass
# keeps within the 8 SQ slots.  Usage: tools/pipes.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-pipes}
shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp COEB_SIDE_STREAM=0
B="python bench.py --pipelines 1 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras $*"
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || echo "rocprofv3 -L rc=$?"
have() { grep -qw "$1" "$out/avail.txt"; }
pass() {
    local name=$1; shift
    local cs=()
    for c in "$@"; do if have "$c"; then cs+=("$c"); else echo "[$name] no counter $c"; fi; done
    [ ${#cs[@]} -eq 0 ] && return 0
    timeout -s KILL 90 rocprofv3 --pmc "${cs[@]}" --kernel-trace --output-format csv -d "$out/$name" -o run -- $B \
        > "$out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc ${cs[*]}"
    [ $rc -ne 0 ] && { tail -n 5 "$out/$name.log"; exit $rc; }
    return 0
}
pass p1 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC
pass p2 SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE
pass p3 SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAVES
pass p4 SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_VMEM SQ_IFETCH SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE
python tools/pmc_summary.py "$out"/p*/run_counter_collection.csv > "$out/summary.txt" 2>&1
grep -E "k_fast|k_describe|k_blur|k_pyr|k_octree|k_match" "$out/summary.txt"
