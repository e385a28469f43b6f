#!/bin/bash
# round 5 session 20: config D's schedule.  The s19 timeline (profiles/r05/s19/timelineD.txt) shows
# k_match_local (one 1024-thread workgroup with ~85 KB of LDS per frame, 0.19 ms alone) stretched
# to 5 ms beside k_pose (256 VGPRs x 4 waves + 62 KB LDS per frame) and the flow kernels.  Knobs:
# stream priorities (COEB_POSE_PRIO / COEB_SIDE_PRIO / COEB_MAIN_PRIO = high|low), the
# local-map matcher reading the frame from global memory (COEB_LOCAL_LDS=0), the shared side stream
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s20
export TMPDIR=/tmp
COEB_LOCAL_LDS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "localmap or batch_track or grab_rgbd" --timeout 120 --timeout-method thread > gpurun_out/s20/pt.log 2>&1
rc=$?; echo "parity (local LDS off) rc=$rc $(tail -1 gpurun_out/s20/pt.log)"; [ $rc -ne 0 ] && exit $rc
run() {   # tag config env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-e2e --no-profile > gpurun_out/s20/$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/s20/$tag.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/s20/$tag.log') if l.startswith('{')][-1]); print('%-22s %s step=%.4f ms value=%.0f' % ('$tag', '$cfg', d['ms_per_step'], d['value']))"
}
for rep in 1 2; do
  run D_base_$rep D X=0
  run D_pose_hi_$rep D COEB_POSE_PRIO=high
  run D_pose_lo_$rep D COEB_POSE_PRIO=low
  run D_local0_$rep D COEB_LOCAL_LDS=0
  run D_local0_pose_hi_$rep D COEB_LOCAL_LDS=0 COEB_POSE_PRIO=high
  run D_shared_$rep D COEB_SIDE_SHARED=1
done
for rep in 1 2; do
  run C_base_$rep C X=0
  run C_shared_$rep C COEB_SIDE_SHARED=1
  run A_base_$rep A X=0
  run A_side_hi_$rep A COEB_SIDE_PRIO=high
  run A_side_lo_$rep A COEB_SIDE_PRIO=low
done
