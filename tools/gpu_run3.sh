set -e
mkdir -p gpurun_out/stamps3
TV_STAMPS=gpurun_out/stamps3/s TV_PROFILE_OUT=gpurun_out/stamps3/ops.json timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-b1 > gpurun_out/stamps3/bench.log 2>&1
python tools/stamps.py gpurun_out/stamps3/s gpurun_out/stamps3/ops.json > gpurun_out/stamps3/summary.txt
grep persistent gpurun_out/stamps3/summary.txt | head -20
