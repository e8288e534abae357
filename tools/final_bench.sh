#!/bin/bash
# Round-end bench lines (the driver's command per config) at the final
# library, after the PMC profiles are committed: profiles/ROUND_bench*.json
#   usage: final_bench.sh ROUND CONFIG...   (CONFIG: c3 | d2 | c2 | c4 | c5)
set -o pipefail
cd $GRAFT_REPO_ROOT
RN=$1; shift
mkdir -p gpurun_out/final
for cfg in "$@"; do
  case $cfg in
    c3) args="" ; out=${RN}_bench ;;
    d2) args="--data d2" ; out=${RN}_bench_c3_d2 ;;
    *)  args="--config $cfg" ; out=${RN}_bench_$cfg ;;
  esac
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 $args > gpurun_out/final/$out.json 2> gpurun_out/final/$out.err || { echo "bench $cfg failed"; tail -5 gpurun_out/final/$out.err; exit 1; }
done
echo done
