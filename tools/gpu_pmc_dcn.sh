# PMC passes restricted to the fused DCN kernel (one DLA34 forward at B=64), plus the counter list.
set -e
O=gpurun_out/pmcdcn; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || echo LIST_FAIL
for s in "a:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "b:SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" "c:TCC_HIT_sum TCC_MISS_sum"; do
  n=${s%%:*}; c=${s#*:}
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex dcn_gemm -d $O -o $n --output-format csv -- python tools/prof_forward.py --iters 1 --model dla34 > $O/$n.log 2>&1 || { echo "PASS_$n FAIL"; tail -5 $O/$n.log; exit 1; }
  echo PASS_$n OK
done
