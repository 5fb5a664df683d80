set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/t_default.log 2>&1 && echo TESTS_OK
for h in 0 1; do
TV_CONV_HALO=$h timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_h$h.log 2>&1
tail -1 gpurun_out/b_h$h.log
done
for a in 1 2 3; do TV_CONV_HALO=0 TV_ABLATE=$a timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_a$a.log 2>&1; tail -1 gpurun_out/b_a$a.log | cut -c1-200; done
