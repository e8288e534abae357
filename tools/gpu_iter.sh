#!/bin/bash
# Iteration run (under gpurun): GPU parity suite, then c3 and c4 benches.
set -o pipefail
O=gpurun_out/iter
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 2
timeout -k 10 240 python bench.py --no-cpu-baseline --no-decode-check --config c4 > $O/c4.json 2> $O/c4.err || exit 3
echo done
