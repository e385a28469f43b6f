#!/bin/bash
# round 5 session 12: k_describe keypoints per wave with the tiled blurred pyramid
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/_kab.sh k_describe main lib/var_kp4.so lib/var_kp16.so main lib/var_kp4.so lib/var_kp16.so
