#!/bin/bash
# round 6 final, part 2: rocprofv3 summaries (A, D), PMC traffic / VALU passes (A, D), timelines,
# the torchrun rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/gpu_session.sh prof profD pmc pmcD timeline timelineD rehearsal
