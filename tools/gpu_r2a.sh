# Round-2 first call: low-precision detection parity (measured drift), GPU suite, bench.
set -e
O=gpurun_out/r2a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TV_PARITY_OUT=$O/parity_lowp.json timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_lowp.py -v --timeout 200 --timeout-method thread > $O/lowp.log 2>&1 || echo LOWP_FAIL
tail -30 $O/lowp.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_parity_lowp.py > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log | cut -c1-1500
