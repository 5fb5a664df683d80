# split-K only for >= 32 k-step layers: conv_lat / schedule / replay tests, B=1 and B=64 lines (R18, DLA-34)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aa; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_lat.py tests/test_gpu_schedule.py tests/test_gpu_replay_b1.py tests/test_gpu_dla34.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 30 > $O/r18_$rep.log 2>&1 || exit 1
  echo "R18 $rep: $(tail -1 $O/r18_$rep.log | grep -o '"value": [0-9.]*') $(tail -1 $O/r18_$rep.log | grep -o '"fp16": {[^}]*}' | grep -o 'ms_per_frame": [0-9.]*')"
  timeout -k 10 300 python bench.py --model dla34 --no-cpu-baseline --no-extras --steps 20 > $O/dla_$rep.log 2>&1 || exit 1
  echo "DLA $rep: $(tail -1 $O/dla_$rep.log | grep -o '"value": [0-9.]*') $(tail -1 $O/dla_$rep.log | grep -o '"fp16": {[^}]*}' | grep -o 'ms_per_frame": [0-9.]*')"
done
