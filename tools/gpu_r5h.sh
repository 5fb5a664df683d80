# conv_burst: GPU tests, then a same-box A/B of the bench line with and without it (TV_BURST=0)
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_conv_burst.py tests/test_gpu_conv_lat.py tests/test_gpu_replay_b1.py tests/test_gpu_schedule.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 > $O/bench_burst.log 2>&1; echo "bench rc=$?"
TV_BURST=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 --allow-env-knobs > $O/bench_noburst.log 2>&1; echo "bench0 rc=$?"
for f in bench_burst bench_noburst; do python -c "
import json,sys; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], {k:v['ms_per_frame'] for k,v in d['latency_b1'].items()}, d['roofline']['per_kernel'].get('tv::lat::conv_lat<_Float16>'), {k:v for k,v in d['roofline']['per_kernel'].items() if 'burst' in k})
"; done
