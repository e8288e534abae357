#!/bin/bash
# Scratch probe (run under gpurun): coder / walk cycle splits alone and
# overlapped, and the c4 GOPs-per-step sweep.
set -o pipefail
mkdir -p gpurun_out/probe
O=gpurun_out/probe


B="python bench.py --no-cpu-baseline --no-decode-check"
timeout -k 10 200 env FFV1HIP_SERIAL=1 FFV1HIP_CODEDBG=1 FFV1HIP_WALKDBG=1 $B --steps 3 > $O/serial.json 2> $O/serial.err || exit 1
timeout -k 10 200 env FFV1HIP_CODEDBG=1 FFV1HIP_WALKDBG=1 $B --steps 3 > $O/over.json 2> $O/over.err || exit 2
for g in 12 16 18; do
  timeout -k 10 300 $B --config c4 --gops $g --steps 5 > $O/c4_$g.json 2> $O/c4_$g.err || exit 3
done
echo done
