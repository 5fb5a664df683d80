set -o pipefail
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_replay_b1.py tests/test_gpu_conv1x1.py tests/test_gpu_schedule.py tests/test_gpu_stem_fuse.py "tests/test_yolact.py::test_gpu_protonet_bench_batch_matches_reference" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $O/tests.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --model yolact --steps 10 --warmup 3 --cpu-seconds 2 > $O/yolact.log 2>&1; echo "yolact rc=$?"; tail -c 1500 $O/yolact.log
