set -e
mkdir -p gpurun_out/stamps4
timeout -k 10 500 python -m pytest tests/test_gpu_forward.py -q -x > gpurun_out/t_fwd.log 2>&1 && echo FWD_OK || { echo FWD_FAIL; tail -30 gpurun_out/t_fwd.log; exit 1; }
TV_PROFILE_OUT=gpurun_out/ops_c3.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1
tail -1 gpurun_out/b_c3.log | cut -c1-300
python tools/opsum.py gpurun_out/ops_c3.json
TV_STAMPS=gpurun_out/stamps4/s TV_PROFILE_OUT=gpurun_out/stamps4/ops.json timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-b1 > gpurun_out/stamps4/bench.log 2>&1
python tools/stamps.py gpurun_out/stamps4/s gpurun_out/stamps4/ops.json > gpurun_out/stamps4/summary.txt
grep persistent gpurun_out/stamps4/summary.txt | head -12 | cut -c1-250
