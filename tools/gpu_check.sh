# Full GPU test suite, then the yolact bench line; outputs under gpurun_out/<tag>/
set -e
O=gpurun_out/${1:-chk}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TV_PARITY_OUT=$O/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAIL|Error|error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline > $O/bench_yolact.log 2>&1 && echo BENCH_OK || { echo BENCH_FAIL; tail -30 $O/bench_yolact.log; exit 1; }
tail -1 $O/bench_yolact.log | cut -c1-1800
