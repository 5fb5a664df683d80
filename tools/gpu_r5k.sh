O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_conv_burst.py tests/test_gpu_conv_lat.py tests/test_gpu_replay_b1.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
for v in 1 0; do
TV_BURST=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 30 --allow-env-knobs > $O/bench_$v.log 2>&1; echo "bench $v rc=$?"
python -c "
import json; d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1])
print('burst=$v', d['value'], d['ms_per_step'], {k:v['ms_per_frame'] for k,v in d['latency_b1'].items()}, {k:v for k,v in d['roofline']['per_kernel'].items() if 'burst' in k or 'lat' in k})
"; done
