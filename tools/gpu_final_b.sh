# Round measurement, part 2 (kernel stats, PMC passes): GPU tests + smoke, the R18 bench line (defaults: CPU baseline, B=1 latency,
# extras), DLA-34 and YOLACT lines, rocprofv3 kernel stats of each, PMC FETCH/WRITE passes (R18 and
# DLA-34 forwards) and the MFMA-utilisation pass. Outputs under gpurun_out/<tag>/. Stops at the
# first step that faults, aborts, segfaults or times out.
TAG=${1:-r3}
O=gpurun_out/$TAG
mkdir -p $O/prof $O/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name"; tail -30 $O/$name.log; exit $rc; fi
  return 0
}
step prof_r18 300 rocprofv3 --kernel-trace --stats -d $O/prof -o r18 --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras
step prof_dla34 300 rocprofv3 --kernel-trace --stats -d $O/prof -o dla34 --output-format csv -- python bench.py --model dla34 --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-extras
step prof_yolact 300 rocprofv3 --kernel-trace --stats -d $O/prof -o yolact --output-format csv -- python bench.py --model yolact --steps 5 --warmup 2 --no-cpu-baseline --no-extras
for m in r18 dla34 yolact; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc/$m -o $c --output-format csv -- python tools/prof_forward.py --iters 1 --model $m > $O/pmc/${m}_$c.log 2>&1
    echo "pmc $m $c rc=$?"
  done
  [ $m = yolact ] && continue
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $O/pmc/$m -o mfma --output-format csv -- python tools/prof_forward.py --iters 1 --model $m > $O/pmc/${m}_mfma.log 2>&1
  echo "pmc $m mfma rc=$?"
done
find $O -name "*.csv" | head -30
