set -e
mkdir -p gpurun_out
for g in 21 24 28 30; do
echo "gops $g" >> gpurun_out/gops.log
timeout -k 10 280 python bench.py --gops $g --steps 10 --no-cpu-baseline --no-decode-check >> gpurun_out/gops.log 2>&1
done
