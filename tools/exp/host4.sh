#!/bin/bash
# host-path rates at 4 hardware queues (the runtime default): tools/exp/host4.sh OUT HOOKS...
# (one bench_host run per FFV1HIP_DEBUG value; "-" = none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
shift
mkdir -p $O
i=0
for h in "$@"; do
  i=$((i + 1))
  [ "$h" = "-" ] && h=""
  FFV1HIP_DEBUG=$h timeout -k 10 400 python -u tools/bench_host.py 20 10 $O/h$i.json > $O/h$i.log 2>&1 || exit $i
done
