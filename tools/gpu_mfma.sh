# MFMA utilisation + held clock per kernel (one PMC pass per model over one B=64 forward).
set -e
O=gpurun_out/${1:-mfma}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in r18 dla34; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $O/$m -o pmc --output-format csv -- python tools/prof_forward.py --iters 1 --model $m > $O/$m.log 2>&1 || { echo "PMC_$m FAIL"; tail -5 $O/$m.log; exit 1; }
  python tools/mfma_util.py $(find $O/$m -name "*counter_collection.csv" | head -n 1) -o $O/mfma_$m.json
done
