# A/B of the in-tree library against a saved variant on the R18 bench workload: GPU parity tests
# of the in-tree build, then per-op HIP-event times (B=64) of both, filtered by kernel name.
#   bash tools/gpu_r18_ab.sh <kernel-name match> <variant> ...
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r18ab; mkdir -p $O
M=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && echo TESTS_OK || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" $O/tests.log | head; exit 1; }
for v in "$@" cur; do
  if [ "$v" = cur ]; then L=""; else L=$PWD/tauv-vision_amd/lib/variants/$v.so; fi
  TV_LIB=$L timeout -k 10 120 python tools/op_bench.py --reps 5 --tag $v > $O/ops_$v.log 2>&1 || { echo "$v OPS_FAIL"; tail $O/ops_$v.log; exit 1; }
  grep -E "$M| total" $O/ops_$v.log | awk -v t=$v '{ if ($2=="total") print; else { s+=$2; n++ } } END { printf "%s %s: %d ops %.4f ms\n", t, "'"$M"'", n, s }'
done
