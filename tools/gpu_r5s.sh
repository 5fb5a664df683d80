# convt3 register-ring body: correctness, then timing of ring depths / schedule barriers
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_convt3.py > $O/t_ct3.log 2>&1
rc=$?; echo "convt3 tests rc=$rc"; grep -E "passed|failed" $O/t_ct3.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/t_ct3.log | head -20; exit $rc; }
run() { timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$1 -o run -- python tools/ct3_time.py $2 > $O/$1.log 2>&1 || { echo "fail $1"; tail -5 $O/$1.log; exit 1; }; }
run base tauv-vision_amd/lib/libtauv_vision_amd.so && timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline --steps 20 > $O/bench_yolact.log 2>&1; echo "bench rc=$?"
tail -c 1500 $O/bench_yolact.log
