# parity + serial and overlapped bench (scratch experiment runner)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
timeout -k 10 200 env FFV1HIP_SERIAL=1 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bs.json 2>gpurun_out/bs.err
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bo.json 2>gpurun_out/bo.err
