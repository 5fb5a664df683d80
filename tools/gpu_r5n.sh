# convt3 (protonet ConvTranspose2d on one halo kernel): single-layer + engine tests, protonet goldens, yolact bench A/B
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_convt3.py > $O/t_ct3.log 2>&1
rc=$?; echo "convt3 tests rc=$rc"; grep -E "passed|failed" $O/t_ct3.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/t_ct3.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_yolact.py -m gpu -k protonet > $O/t_yol.log 2>&1
rc=$?; echo "yolact tests rc=$rc"; grep -E "passed|failed" $O/t_yol.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAIL|Error|error" $O/t_yol.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model yolact --no-cpu-baseline --steps 20 > $O/bench_yolact.log 2>&1; echo "bench rc=$?"
tail -c 3000 $O/bench_yolact.log
