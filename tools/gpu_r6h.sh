O=gpurun_out/r6h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipe_split.py tests/test_gpu_api_graph.py -m gpu > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -5 $O/tests.log
[ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for cfg in "0 16" "1 4" "1 8" "1 16" "1 32"; do set -- $cfg
  for m in r18 dla34; do
    TV_PIPE_SPLIT=$1 TV_PIPE_SPLIT_MAX=$2 OPS_MODEL=$m timeout -k 10 200 python tools/b1_ops.py fp32 1 > $O/ops_${m}_$1_$2.log 2>&1 || exit 3
    echo "$m split=$1 max=$2: $(head -3 $O/ops_${m}_$1_$2.log | tr '\n' ' ')"
  done
done
