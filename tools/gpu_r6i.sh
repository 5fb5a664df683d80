# conv_pipe split-K: tests, fp32 B=1 sweep of the hand-off cost / slice cap, R18 bench line (fp32 leg, node leg)
O=gpurun_out/r6i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipe_split.py tests/test_gpu_forward.py -m gpu > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/tests.log
[ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for cfg in "1 16 5" "1 16 3" "1 16 8" "1 32 5" "1 8 5"; do set -- $cfg
  for m in r18 dla34; do
    TV_PIPE_SPLIT=$1 TV_PIPE_SPLIT_MAX=$2 TV_PIPE_SPLIT_RED=$3 OPS_MODEL=$m timeout -k 10 200 python tools/b1_ops.py fp32 1 $O/ops_${m}_$2_$3.json > $O/ops_${m}_$2_$3.log 2>&1 || exit 3
    echo "$m max=$2 red=$3: $(grep -v amdgpu.ids $O/ops_${m}_$2_$3.log | head -4 | tr '\n' ' ')"
  done
done
timeout -k 10 500 python bench.py > $O/bench_r18.log 2>&1 || exit 4
tail -1 $O/bench_r18.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r18', d['value'], d['ms_per_step'], 'fp32', d.get('fp32_value'), 'node', d.get('node_b1'), 'api', d.get('api'))"
