# level-grouped launches on the 32-frame slices too (knob TV_LATGROUP_B=32) at B=64, R18 and DLA-34, interleaved
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ac; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_LATGROUP_B=32"; do
    n=$(echo "${k:-default}" | tr ' =' '__')
    env $k timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 30 > $O/r18_${rep}_$n.log 2>&1 || { echo "FAIL r18 $k"; tail -3 $O/r18_${rep}_$n.log; exit 1; }
    echo "rep $rep R18 ${k:-default}: $(tail -1 $O/r18_${rep}_$n.log | grep -o '"value": [0-9.]*')"
    env $k timeout -k 10 300 python bench.py --model dla34 --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 20 > $O/dla_${rep}_$n.log 2>&1 || { echo "FAIL dla $k"; exit 1; }
    echo "rep $rep DLA ${k:-default}: $(tail -1 $O/dla_${rep}_$n.log | grep -o '"value": [0-9.]*')"
  done
done
