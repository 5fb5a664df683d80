# Decode rewrite + parity + suite + bench (round 2)
set -e
O=gpurun_out/r2b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -v --timeout 120 --timeout-method thread > $O/decode.log 2>&1 && echo DECODE_OK || { echo DECODE_FAIL; tail -50 $O/decode.log; exit 1; }
TV_PARITY_OUT=$O/parity_lowp.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && echo BENCH_OK || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-3000
