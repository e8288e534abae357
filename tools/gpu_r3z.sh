#!/bin/bash
# Round 3: GPU suite on the cleaned library (split-walk hook without the
# share knob); walk wave priority 1 / 2 under the range pass's 3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
for v in w0 w1 w2; do
  case $v in
    w0) E="" ;;
    w1) E="FFV1HIP_WALK_PRIO=1" ;;
    w2) E="FFV1HIP_WALK_PRIO=2" ;;
  esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
