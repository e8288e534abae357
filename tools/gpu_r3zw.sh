#!/bin/bash
# Round 3: gpu_r3z.sh (GPU suite, walk priority) then gpu_r3w.sh (configs,
# two-rank launch on one device, host rates).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3z.sh || exit $?
bash tools/gpu_r3w.sh || exit $((10 + $?))
