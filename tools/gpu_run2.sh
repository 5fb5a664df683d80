set -e
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_forward.py -q -x > gpurun_out/t_fwd.log 2>&1 && echo FWD_OK || { echo FWD_FAIL; tail -30 gpurun_out/t_fwd.log; exit 1; }
TV_PROFILE_OUT=gpurun_out/ops_c3.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_c3.log 2>&1
tail -1 gpurun_out/b_c3.log | cut -c1-600
python tools/opsum.py gpurun_out/ops_c3.json
