# A/B of library builds on per-kernel times of one bench slice (tools/kern_ab.py), interleaved
# twice to see box drift: bash tools/gpu_libab.sh <tag> <libdir>... ("lib" = the in-tree build)
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for L in "$@"; do
    TV_LIB=$GRAFT_REPO_ROOT/tauv-vision_amd/$L/libtauv_vision_amd.so timeout -k 10 120 python tools/kern_ab.py --model ${MODEL:-r18} --tag "$L.$rep" --ops $O/ops_$L.$rep.json >> $O/ab.jsonl 2> $O/err_$L.log
    rc=$?
    echo "$L.$rep rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $O/err_$L.log; exit $rc; fi
  done
done
python - $O/ab.jsonl <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
names = sorted({k for r in rows for k in r["kernels"]}, key=lambda k: -rows[0]["kernels"].get(k, {"ms": 0})["ms"])
print("%-62s" % "kernel" + "".join("%12s" % r["tag"][:11] for r in rows))
print("%-62s" % "TOTAL" + "".join("%12.4f" % r["total_ms"] for r in rows))
for k in names[:14]:
    print("%-62s" % k[:62] + "".join("%12.4f" % r["kernels"].get(k, {"ms": float("nan")})["ms"] for r in rows))
EOF
