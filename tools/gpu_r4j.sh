# round 4: stem_s2 cycle stamps (stamp build lib_s9) + the YOLACT PMC traffic passes
O=gpurun_out/r4j
mkdir -p $O/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S9=$GRAFT_REPO_ROOT/tauv-vision_amd/lib_s9/libtauv_vision_amd.so
TV_LIB=$S9 timeout -k 10 200 python tools/c3_stamps.py --match block_layers.0.conv1 --kernel tv::ss2:: > $O/ss2_stamps.json 2> $O/stamps.err || exit $?
TV_LIB=$S9 timeout -k 10 200 python tools/c3_stamps.py --match block_layers.0.conv2 > $O/c3_b0c2_stamps.json 2>> $O/stamps.err || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc/yolact -o $c --output-format csv -- python tools/prof_forward.py --iters 1 --model yolact > $O/pmc/yolact_$c.log 2>&1 || exit $?
done
find $O -name "*.csv" | head
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_yolact.py -m gpu > $O/test_yolact.log 2>&1 || { tail -30 $O/test_yolact.log; exit 1; }
tail -1 $O/test_yolact.log
timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline > $O/bench_yolact.log 2>&1 || exit $?
tail -1 $O/bench_yolact.log | cut -c1-600
