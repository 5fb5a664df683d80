# per-kernel A/B (in-tree build vs another) for YOLACT and DLA-34, then their bench lines:
# bash tools/gpu_models_ab.sh <tag> <libdir>
TAG=$1; ALT=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
MODEL=yolact timeout -k 10 300 bash tools/gpu_libab.sh $TAG/ab_yolact lib $ALT > $O/ab_yolact.log 2>&1; rc=$?; echo "ab yolact rc=$rc"; tail -12 $O/ab_yolact.log
if [ $rc -ne 0 ]; then exit $rc; fi
for M in yolact dla34; do
  timeout -k 10 400 python bench.py --model $M --no-cpu-baseline > $O/bench_$M.log 2>&1; rc=$?; echo "bench $M rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/bench_$M.log; exit $rc; fi
  tail -1 $O/bench_$M.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('latency_b1'))"
done
