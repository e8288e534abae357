#!/bin/bash
# Round 3: per-wave walk trace (start spread, run time, end) of the c3 bench,
# overlapped (default) and alone (FFV1HIP_SERIAL), and one records set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3j
mkdir -p $O
FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 8 > $O/tr_def.json 2> $O/tr_def.err || exit 1
FFV1HIP_WALKTRACE=1 FFV1HIP_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 4 > $O/tr_serial.json 2> $O/tr_serial.err || exit 2
FFV1HIP_WALKTRACE=1 FFV1HIP_RECSETS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 8 > $O/tr_rec1.json 2> $O/tr_rec1.err || exit 3

for g in 16 18 24 28; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 8 --gops $g > $O/gops_$g.json 2> $O/gops_$g.err || exit 4
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 8 > $O/gops_21.json 2> $O/gops_21.err || exit 5
echo done2
