#!/bin/bash
# One parametrised GPU job (under gpurun): steps chained, each with its own
# time limit; the first failure ends the job.
#   tools/gpu_run.sh OUT STEP...      STEP is one of:
#     tests                 the -m gpu suite (+ smoke())
#     bench[:ARGS]          bench.py ARGS (default: the driver's command)
#     serial[:ARGS]         bench.py with FFV1HIP_DEBUG=serial (kernels one at a time)
#     prof:TAG[:ARGS]       tools/profile_round.sh TAG ARGS (rocprof stats + PMC)
#     env:NAME=VAL          set an environment variable for the later steps
#     py:SCRIPT[:ARGS]      python SCRIPT ARGS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
shift
mkdir -p "$O"
n=0
for s in "$@"; do
  n=$((n + 1))
  kind=${s%%:*}
  rest=${s#*:}
  [ "$rest" = "$s" ] && rest=""
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit $n
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $n ;;
    bench)
      timeout -k 10 600 python bench.py ${rest:---gpus 1 --steps 20 --warmup 5} > $O/bench$n.json 2> $O/bench$n.err || exit $n ;;
    serial)
      FFV1HIP_DEBUG=serial${FFV1HIP_DEBUG:+,$FFV1HIP_DEBUG} timeout -k 10 600 python bench.py --no-cpu-baseline ${rest:---steps 5} > $O/serial$n.json 2> $O/serial$n.err || exit $n ;;
    prof)
      tag=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 1100 bash tools/profile_round.sh $tag $args > $O/prof$n.log 2>&1 || exit $n ;;
    env)
      export "$rest" ;;
    py)
      scr=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 600 python -u $scr $args > $O/py$n.log 2>&1 || exit $n ;;
    *) echo "unknown step $s"; exit 99 ;;
  esac
done
echo done
