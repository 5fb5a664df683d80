# YOLACT GPU tests + bench line + NMS kernel times (rocprofv3 stats of a short bench)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ycheck}; mkdir -p $O/prof
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_yolact.py -m gpu > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" $O/tests.log | tail -3
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('mask_roofline'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o y --output-format csv -- python bench.py --model yolact --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/prof.log 2>&1; echo "prof rc=$?"
grep -E "nms|rocprim|assemble" $O/prof/y_kernel_stats.csv | cut -c1-160
