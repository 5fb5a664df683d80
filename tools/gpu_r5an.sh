# stem_conv NI=1 (DLA-34 base layer) with one E buffer, two workgroups per CU: tests, kernel time, bench
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dla34.py tests/test_gpu_stem_fuse.py tests/test_gpu_forward.py tests/test_gpu_replay_b1.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --model dla34 --no-cpu-baseline --no-extras --no-b1 --steps 5 --warmup 2 > $O/prof.log 2>&1 || { echo "PROF FAIL"; exit 1; }
grep -i "stem_conv\|conv_small" $O/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
for rep in 1 2; do
  timeout -k 10 300 python bench.py --model dla34 --no-cpu-baseline --no-extras > $O/dla_$rep.log 2>&1 || { echo "FAIL"; exit 1; }
  echo "rep $rep: $(tail -1 $O/dla_$rep.log | grep -o '"value": [0-9.]*\|ms_per_frame": [0-9.]*' | tr '\n' ' ')"
done
