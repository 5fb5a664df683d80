# One full measurement call: GPU tests, smoke, bench line, rocprofv3 kernel stats of the bench,
# PMC passes (FETCH_SIZE / WRITE_SIZE) over one forward. Outputs under gpurun_out/<tag>/.
set -e
TAG=${1:-r1}
O=gpurun_out/$TAG
mkdir -p $O/prof $O/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo SMOKE_OK
BENCH_PROFILE_OUT=$O/ops.json timeout -k 10 400 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rprof --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras > $O/prof.log 2>&1
# PMC passes: one forward of the bench workload (B=64 u8 frames = two concurrent 32-frame slices)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc -o $c --output-format csv -- python tools/prof_forward.py --iters 1 > $O/pmc/$c.log 2>&1
done
find $O -name "*.csv" | head -20
