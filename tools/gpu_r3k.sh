#!/bin/bash
# Round 3: walk trace + GOP sweep (tools/gpu_r3j.sh), then the host-path
# timing breakdown (tools/gpu_r3i.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r3j.sh || exit 1
bash tools/gpu_r3i.sh || exit 2
echo done
