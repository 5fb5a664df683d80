# final round-5 state: GPU tests + smoke, DLA-34 line, its kernel stats and HBM traffic
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aq; mkdir -p $O/prof $O/pmc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
BENCH_PROFILE_OUT=$O/ops_dla34.json timeout -k 10 300 python bench.py --model dla34 --cpu-seconds 10 > $O/bench_dla34.log 2>&1 || { tail -20 $O/bench_dla34.log; exit 1; }
tail -1 $O/bench_dla34.log | grep -o '"value": [0-9.]*\|ms_per_frame": [0-9.]*' | tr '\n' ' '; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o dla34 --output-format csv -- python bench.py --model dla34 --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras > $O/prof.log 2>&1 || { echo PROF FAIL; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc/dla34 -o $c --output-format csv -- python tools/prof_forward.py --iters 1 --model dla34 > $O/pmc/dla34_$c.log 2>&1 || { echo "PMC FAIL $c"; exit 1; }
done
echo done
