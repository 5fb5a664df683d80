# PMC counter passes over one forward of the bench workload (kernel-level counters).
set -e
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for s in "a:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "b:SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "c:TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  n=${s%%:*}; c=${s#*:}
  timeout -k 10 240 rocprofv3 --pmc $c -d gpurun_out/pmc2 -o $n --output-format csv -- python tools/prof_forward.py --iters 1 > gpurun_out/pmc2/$n.log 2>&1
done
ls gpurun_out/pmc2
