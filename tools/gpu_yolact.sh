set -e
O=gpurun_out/r2b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_yolact.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/yolact.log 2>&1 && echo YOLACT_OK || { echo YOLACT_FAIL; tail -40 $O/yolact.log; exit 1; }
