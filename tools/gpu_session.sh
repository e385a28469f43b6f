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
SIDE0=${COEB_SIDE_STREAM-unset}
for step in "$@"; do
    # the PMC steps export COEB_SIDE_STREAM=0 for their passes: restore the caller's setting per step
    if [ "$SIDE0" = unset ]; then unset COEB_SIDE_STREAM; else export COEB_SIDE_STREAM=$SIDE0; fi
    case "$step" in
        pytest) run pytest_gpu 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread ;;
        scale) run scale 900 python -u -m pytest tests/test_gpu_bench_scale.py -v -s -m gpu --timeout 300 --timeout-method thread ;;
        pytestall) run pytest_gpu 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ;;
        smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 600 python bench.py ;;
        benchB) run benchB 600 python bench.py --config B --batch 64 --no-cpu-baseline ;;
        benchC) run benchC 600 python bench.py --config C --no-cpu-baseline --no-extras ;;
        benchD) run benchD 600 python bench.py --config D --no-cpu-baseline --no-extras ;;
        # per-kernel evidence with the side stream off and one pipeline: every kernel is then one
        # whole-batch launch running alone, the same launches bench.py's HIP-event pass times (it
        # disables the side stream and profiles pipeline 0 by itself)
        prof) COEB_SIDE_STREAM=0 run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --pipelines 1 --batch 1024 --no-cpu-baseline --no-e2e --no-extras ;;
        profD) COEB_SIDE_STREAM=0 run profD 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profD -o run -- python bench.py --config D --no-cpu-baseline --no-e2e --no-extras --steps 5 --warmup 2 ;;
        diag) run diag 600 python tools/diag_parity.py ;;
        # kernel timeline of the default two-pipeline step (concurrency / idle time per step)
        timeline)
            run timeline 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile
            python tools/timeline2.py gpurun_out/tl/run_kernel_trace.csv 3 > gpurun_out/timeline.txt 2>&1; tail -n 30 gpurun_out/timeline.txt ;;
        timelineD)
            run timelineD 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlD -o run -- python bench.py --config D --steps 4 --warmup 2 --no-cpu-baseline --no-extras --no-e2e --no-profile
            python tools/timeline2.py gpurun_out/tlD/run_kernel_trace.csv 2 > gpurun_out/timelineD.txt 2>&1; tail -n 30 gpurun_out/timelineD.txt ;;
        rehearsal)
            # the process-per-GPU path (torch.distributed.run, gloo barrier / max) with both ranks on
            # device 0 of this one-GPU box: plumbing only, the line is marked rehearsal_one_device
            COEB_BENCH_ONE_DEVICE=1 run rehearsal 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-e2e ;;
        posetime) run posetime 300 python tools/pose_timing.py ;;
        flow) run flow 300 python tools/flow_bench.py ;;
        flowprof) run flowprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/flowprof -o run -- python tools/flow_bench.py ;;
        pmc)
            export COEB_SIDE_STREAM=0
            B="python bench.py --pipelines 1 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
            run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- $B
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv \
                --json gpurun_out/pmc_traffic.json --frames 1025 --command "$B" > gpurun_out/pmc_traffic.log 2>&1
            run pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- $B
            run pmc_sq2 600 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq2 -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmc_sq/run_counter_collection.csv gpurun_out/pmc_sq2/run_counter_collection.csv \
                --valu-json gpurun_out/pmc_valu.json --frames 1025 --command "$B" > gpurun_out/pmc_valu.log 2>&1
            ;;
        pmcB)
            export COEB_SIDE_STREAM=0
            # config B: 512 frames as two pipelines, launches of 257 frames (256 + the halo frame)
            B="python bench.py --config B --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
            run pmcB_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcB_fetch -o run -- $B
            run pmcB_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcB_write -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmcB_fetch/run_counter_collection.csv gpurun_out/pmcB_write/run_counter_collection.csv \
                --json gpurun_out/pmc_traffic_1280x960.json --frames 257 --size 1280x960 --command "$B" > gpurun_out/pmcB_traffic.log 2>&1
            run pmcB_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmcB_sq -o run -- $B
            run pmcB_sq2 600 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcB_sq2 -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmcB_sq/run_counter_collection.csv gpurun_out/pmcB_sq2/run_counter_collection.csv \
                --valu-json gpurun_out/pmc_valu_1280x960.json --frames 257 --size 1280x960 --command "$B" > gpurun_out/pmcB_valu.log 2>&1
            ;;
        benchB512) run benchB512 600 python bench.py --config B ;;
        benchCfull) run benchC 600 python bench.py --config C ;;
        benchDfull) run benchD 600 python bench.py --config D --no-extras ;;
        pmcD)
            # the configs[4] loop's kernels (flow, pose, TrackLocalMap) with their own traffic / VALU passes
            export COEB_SIDE_STREAM=0
            # two 512-frame pipelines: launches of 515 frames (512 + the 3-frame halo; round 5 fixed the
            # stale 259 that scaled the D line's traffic)
            B="python bench.py --config D --pipelines 2 --batch 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-e2e --no-extras"
            run pmcD_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcD_fetch -o run -- $B
            run pmcD_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcD_write -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmcD_fetch/run_counter_collection.csv gpurun_out/pmcD_write/run_counter_collection.csv \
                --json gpurun_out/pmc_traffic_D.json --frames 515 --command "$B" > gpurun_out/pmcD_traffic.log 2>&1
            run pmcD_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmcD_sq -o run -- $B
            run pmcD_sq2 600 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcD_sq2 -o run -- $B
            python tools/pmc_summary.py gpurun_out/pmcD_sq/run_counter_collection.csv gpurun_out/pmcD_sq2/run_counter_collection.csv \
                --valu-json gpurun_out/pmc_valu_D.json --frames 515 --command "$B" > gpurun_out/pmcD_valu.log 2>&1
            ;;
        *) echo "unknown step $step" ;;
    esac
done
