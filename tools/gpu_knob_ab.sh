# GPU tests, then a per-kernel A/B (tools/kern_ab.py, two interleaved reps) of the default engine
# against one diagnostic knob setting, then the bench line: bash tools/gpu_knob_ab.sh <tag> KNOB=V
TAG=$1; KNOB=$2
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; tail -30 $O/$name.log; exit $rc; fi
  return 0
}
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu ${TESTS:-}
grep -E "passed|failed|FAILED" $O/tests.log | tail -4
for rep in 1 2; do
  step ab_def_$rep 120 python tools/kern_ab.py --model ${MODEL:-r18} --tag def.$rep
  cat $O/ab_def_$rep.log | tail -1 >> $O/ab.jsonl
  env $KNOB timeout -k 10 120 python tools/kern_ab.py --model ${MODEL:-r18} --tag knob.$rep > $O/ab_knob_$rep.log 2>&1; echo "knob.$rep rc=$?"
  cat $O/ab_knob_$rep.log | tail -1 >> $O/ab.jsonl
done
python - $O/ab.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
names = sorted({k for r in rows for k in r["kernels"]}, key=lambda k: -rows[0]["kernels"].get(k, {"ms": 0})["ms"])
print("%-64s" % "kernel" + "".join("%10s" % r["tag"][:9] for r in rows))
print("%-64s" % "TOTAL" + "".join("%10.4f" % r["total_ms"] for r in rows))
for k in names[:16]:
    print("%-64s" % k[:64] + "".join("%10.4f" % r["kernels"].get(k, {"ms": float("nan")})["ms"] for r in rows))
PY
BENCH_PROFILE_OUT=$O/ops_r18.json step bench 400 python bench.py --model ${MODEL:-r18} --no-cpu-baseline --no-b1
tail -1 $O/bench.log | cut -c1-600
env $KNOB timeout -k 10 400 python bench.py --model ${MODEL:-r18} --no-cpu-baseline --no-b1 --allow-env-knobs --no-extras > $O/bench_knob.log 2>&1; echo "bench_knob rc=$?"
tail -1 $O/bench_knob.log | cut -c1-300
