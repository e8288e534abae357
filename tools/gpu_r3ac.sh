#!/bin/bash
# Round 3: the longer plane group's walk waves one / two priority levels up.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ac
mkdir -p $O
run() {  # tag env args...
  local tag=$1 env=$2; shift 2
  env $env timeout -k 10 400 python bench.py --no-cpu-baseline --no-decode-check "$@" > $O/b_$tag.json 2> $O/b_$tag.err
}
run c3_b0 "" --steps 20 || exit 1
run c3_b1 "FFV1HIP_WALK_LONG_BOOST=1" --steps 20 || exit 2
run c3_b2 "FFV1HIP_WALK_LONG_BOOST=2" --steps 20 || exit 3
run c4_b0 "" --config c4 --steps 10 || exit 4
run c4_b1 "FFV1HIP_WALK_LONG_BOOST=1" --config c4 --steps 10 || exit 5
run c5_b1 "FFV1HIP_WALK_LONG_BOOST=1" --config c5 --steps 10 || exit 6
run c2_b1 "FFV1HIP_WALK_LONG_BOOST=1" --config c2 --steps 10 || exit 7
echo done
