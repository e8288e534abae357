#!/bin/bash
# Full -m gpu suite then a short bench (run under gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 10 > gpurun_out/bench_check.log 2>&1 || exit 2
echo done
