#!/bin/bash
# Round profiles (under gpurun): rocprof kernel stats + PMC HBM traffic for c3 and c4.
set -o pipefail
bash tools/profile_round.sh r02 --steps 5 || exit 1
bash tools/profile_round.sh r02_c4 --config c4 --steps 5 || exit 2
echo done
