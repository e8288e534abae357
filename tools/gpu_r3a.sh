#!/bin/bash
# Round 3, first box: the new parity tests first, then the whole -m gpu
# suite, smoke(), the c3 bench (every GOP against the oracle fixture) and the
# two-rank launcher rehearsal on one device.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3a
O=gpurun_out/r3a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "never_truncates or full_size" > $O/new.log 2>&1 || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 4
FFV1_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --gops 6 --steps 5 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err || exit 5
echo done
