# YOLACT slices A/B (B=32: 2 x 16 default, 1 x 32, 4 x 8), interleaved twice
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ad; mkdir -p $O
for rep in 1 2; do
  for k in "" "TV_SLICES=1" "TV_SLICES=4"; do
    n=$(echo "${k:-default}" | tr ' =' '__')
    env $k timeout -k 10 300 python bench.py --model yolact --allow-env-knobs --no-cpu-baseline --no-extras --steps 30 > $O/y_${rep}_$n.log 2>&1 || { echo "FAIL $k"; tail -3 $O/y_${rep}_$n.log; exit 1; }
    echo "rep $rep ${k:-default}: $(tail -1 $O/y_${rep}_$n.log | grep -o '"value": [0-9.]*')"
  done
done
