#!/bin/bash
# c5 GOPs per step with the split schedule (under gpurun).
set -o pipefail
O=gpurun_out/c5g
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check --config c5"
for g in 5 6 7; do
  timeout -k 10 300 $B --gops $g > $O/g$g.json 2> $O/g$g.err || exit 1
done
echo done
