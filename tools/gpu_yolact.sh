# YOLACT GPU tests + the yolact bench line (+ rocprofv3 kernel stats of it)
set -e
O=gpurun_out/${1:-r2b}; mkdir -p $O/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_yolact.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/yolact.log 2>&1 && echo YOLACT_OK || { echo YOLACT_FAIL; tail -40 $O/yolact.log; exit 1; }
timeout -k 10 300 python bench.py --model yolact --cpu-seconds 5 > $O/bench_yolact.log 2>&1 && echo BENCH_OK || { echo BENCH_FAIL; tail -30 $O/bench_yolact.log; exit 1; }
tail -1 $O/bench_yolact.log | cut -c1-1500
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o rprof_yolact --output-format csv -- python bench.py --model yolact --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_yolact.log 2>&1 && echo PROF_OK
