#!/bin/bash
# Round 3: gpu_r3ac.sh (longer plane group's walk priority) then
# gpu_r3ad.sh (rocprof + PMC of c2, c4, c5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3ac.sh || exit $?
bash tools/gpu_r3ad.sh || exit $((10 + $?))
