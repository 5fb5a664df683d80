O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 30 > $O/bench.log 2>&1; echo "bench rc=$?"
python -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k:v['ms_per_frame'] for k,v in d['latency_b1'].items()}, d['roofline']['frac'], d['roofline']['per_kernel'].get('tv::c3::conv3x3<_Float16, _Float16, 32, 2, 1, 0, 4, 4, 8>'))
"
