#!/bin/bash
# Round 3, final library: gpu_r3ah.sh (D2 content, two-rank rehearsal) then
# gpu_r3ai.sh (side grids).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3ah.sh || exit $?
bash tools/gpu_r3ai.sh || exit $((10 + $?))
