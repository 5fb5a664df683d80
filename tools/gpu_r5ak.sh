# conv_small LDS-halo variant: tests, DLA-34 B=64 A/B, per-kernel times
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ak; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_small.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for h in 0 1; do
    TV_CSM_HALO=$h timeout -k 10 300 python bench.py --model dla34 --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 20 > $O/dla_${rep}_$h.log 2>&1 || { echo "FAIL $h"; exit 1; }
    echo "rep $rep halo $h: $(tail -1 $O/dla_${rep}_$h.log | grep -o '"value": [0-9.]*')"
  done
done
for h in 0 1; do
  TV_CSM_HALO=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$h -o run -- python bench.py --model dla34 --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 5 --warmup 2 > $O/prof_$h.log 2>&1 || { echo "PROF FAIL $h"; exit 1; }
  f=$(find $O/prof_$h -name '*kernel_stats.csv' | head -1)
  echo "halo $h:"; grep -i "conv_small" $f | cut -d, -f1-4 | cut -c1-200
done
