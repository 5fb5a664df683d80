# A/B of fused-DCN variants: parity of each variant on the DLA34 tests, then per-op DLA34 times
#   bash tools/gpu_dcn_ab.sh <variant> ...   (tauv-vision_amd/lib/variants/<variant>.so; "cur" = in-tree)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dcnab; mkdir -p $O
for v in "$@"; do
  if [ "$v" = cur ]; then L=""; else L=$PWD/tauv-vision_amd/lib/variants/$v.so; fi
  TV_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_dla34.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1 && echo "$v TESTS_OK" || { echo "$v TESTS_FAIL"; grep -E "FAILED|Error|assert" $O/t_$v.log | head; exit 1; }
  TV_LIB=$L OPS_MODEL=dla34 timeout -k 10 120 python tools/b1_ops.py fp16 64 $O/ops_$v.json > $O/ops_$v.log 2>&1 || { echo "$v OPS_FAIL"; tail $O/ops_$v.log; exit 1; }
  python - $O/ops_$v.json $v <<'PY'
import json, sys
ops = json.load(open(sys.argv[1]))
d = [o for o in ops if "dcn" in o["kernel"]]
print(sys.argv[2], "total %.3f ms  dcn %.3f ms" % (sum(o["ms"] for o in ops), sum(o["ms"] for o in d)))
for o in d: print("   %7.3f ms %6.1f TF %s" % (o["ms"], o["gflop"] / o["ms"], o["op"][:50]))
PY
done
