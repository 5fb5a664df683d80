# convt3 PMC passes over tools/ct3_time.py (per-dispatch counters of the 138x138 layer)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r5r; mkdir -p $O
for s in "a:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "b:SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
         "c:FETCH_SIZE" "d:WRITE_SIZE"; do
  n=${s%%:*}; c=${s#*:}
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex convt3 -d $O/pmc -o $n --output-format csv -- python tools/ct3_time.py > $O/pmc_$n.log 2>&1 || { echo "PMC_$n FAIL"; tail -5 $O/pmc_$n.log; exit 1; }
done
echo PMC_OK
