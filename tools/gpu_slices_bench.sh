# R18 bench line at TV_SLICES = 2 (default), 1, 3, 4, then 2 again (box drift):
# bash tools/gpu_slices_bench.sh <tag>
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in 2 1 3 4 2; do
  TV_SLICES=$k timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-b1 --no-extras > $O/bench_s$k.log 2>&1; rc=$?
  echo "slices $k rc=$rc $(tail -1 $O/bench_s$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  if [ $rc -ne 0 ]; then tail -5 $O/bench_s$k.log; exit $rc; fi
done
