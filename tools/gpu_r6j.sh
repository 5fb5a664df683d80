# conv_lat<float> on the fp32 path: tests, fp32 B=1 per-op sweep of its split cap, R18 bench line
O=gpurun_out/r6j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipe_split.py tests/test_gpu_forward.py tests/test_gpu_dla34.py tests/test_gpu_api_graph.py -m gpu > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -3 $O/tests.log
[ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for cfg in 8 4 16; do
  for m in r18 dla34; do
    TV_LAT_SPLIT_F32=$cfg OPS_MODEL=$m timeout -k 10 200 python tools/b1_ops.py fp32 1 $O/ops_${m}_$cfg.json > $O/ops_${m}_$cfg.log 2>&1 || exit 3
    echo "$m lat_split_f32=$cfg: $(grep -v amdgpu.ids $O/ops_${m}_$cfg.log | head -5 | tr '\n' ' ')"
  done
done
timeout -k 10 500 python bench.py > $O/bench_r18.log 2>&1 || exit 4
tail -1 $O/bench_r18.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r18', d['value'], d['ms_per_step'], 'fp32', d.get('fp32_value'), 'node', d.get('node_b1'), 'b1', {k: v['ms_per_frame'] for k, v in (d.get('latency_b1') or {}).items()})"
