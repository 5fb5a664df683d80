# Quick check of a kernel change: all GPU tests, then the three bench lines (no CPU baseline,
# extras or B=1 legs) with per-op HIP-event times. Outputs under gpurun_out/<tag>/.
set -e
O=gpurun_out/${1:-ab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
for m in r18 dla34 yolact; do
  BENCH_PROFILE_OUT=$O/ops_$m.json timeout -k 10 300 python bench.py --model $m --no-cpu-baseline --no-extras --no-b1 > $O/bench_$m.log 2>&1 || { echo "BENCH_$m FAIL"; tail -5 $O/bench_$m.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$m.log').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
