#!/bin/bash
# c4 GOPs-per-step sweep (under gpurun).
set -o pipefail
O=gpurun_out/gops
mkdir -p $O
for g in 14 16 17; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --config c4 --gops $g > $O/c4_$g.json 2> $O/c4_$g.err || exit 1
done
for g in 24 28; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --gops $g > $O/c3_$g.json 2> $O/c3_$g.err || exit 1
done
echo done
