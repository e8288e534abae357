#!/bin/bash
# Round profiles (under gpurun): the default bench line and, on the same box,
# rocprof kernel stats + PMC HBM traffic of the same bench command (c3), then c4.
set -o pipefail
mkdir -p gpurun_out/benches
timeout -k 10 400 python bench.py > gpurun_out/benches/c3.json 2> gpurun_out/benches/c3.err || exit 1
bash tools/profile_round.sh r02 || exit 2
bash tools/profile_round.sh r02_c4 --config c4 --steps 10 || exit 3
echo done
