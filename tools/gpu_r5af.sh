# within-box spread of the R18 bench line: 4 back-to-back default-config runs (no CPU baseline / extras)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5af; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 20 > $O/r18_$i.log 2>&1 || { echo "FAIL $i"; exit 1; }
  echo "run $i: $(tail -1 $O/r18_$i.log | grep -o '"value": [0-9.]*') $(tail -1 $O/r18_$i.log | grep -o '"eager_value": [0-9.]*') $(tail -1 $O/r18_$i.log | grep -o '"frac": [0-9.]*' | head -1)"
done
for rep in 1 2; do
  for k in "TV_C3_HALF_COST=0" "TV_C3_HALF_COST=70" "TV_C3_NW=8" ""; do
    n=$(echo "${k:-default}" | tr ' =' '__')
    env $k timeout -k 10 300 python bench.py --allow-env-knobs --no-cpu-baseline --no-extras --no-b1 --steps 20 > $O/k_${rep}_$n.log 2>&1 || { echo "FAIL $k"; exit 1; }
    echo "rep $rep ${k:-default}: $(tail -1 $O/k_${rep}_$n.log | grep -o '"value": [0-9.]*')"
  done
done
