#!/bin/bash
# Round 3: rocprof kernel stats + PMC FETCH/WRITE for c2, c4, c5 (their
# bench lines' roofline traffic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in c2 c4 c5; do
  timeout -k 10 900 bash tools/profile_round.sh r03_$c --config $c --steps 3 --no-decode-check > gpurun_out/prof_r03_$c.log 2>&1 || exit 1
done
echo done
