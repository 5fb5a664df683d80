# One profiling call: GPU tests, the full bench line, rocprofv3 kernel stats of the bench,
# and the two PMC passes for HBM traffic. Outputs under gpurun_out/.
set -e
mkdir -p gpurun_out/prof gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1 && echo TESTS_OK
TV_PROFILE_OUT=gpurun_out/ops.json timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o rprof --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b1 > gpurun_out/prof.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmc -o $c --output-format csv -- python tools/prof_forward.py --iters 1 > gpurun_out/pmc/$c.log 2>&1
done
ls gpurun_out/prof gpurun_out/pmc
mkdir -p gpurun_out/stamps
TV_STAMPS=gpurun_out/stamps/s TV_PROFILE_OUT=gpurun_out/stamps/ops.json timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-b1 > gpurun_out/stamps/bench.log 2>&1
python tools/stamps.py gpurun_out/stamps/s gpurun_out/stamps/ops.json > gpurun_out/stamps/summary.txt
head -30 gpurun_out/stamps/summary.txt
