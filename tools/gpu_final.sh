#!/bin/bash
# Round-end rehearsal (under gpurun): the -m gpu suite, smoke(), the default bench.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
