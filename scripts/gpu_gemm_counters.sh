# Counter passes over bench/gemm_counters.py (kernel trace only, never with sys/runtime traces),
# GCTR=decode (default) or prefill.  One rocprofv3 run per pass, each within the per-block limits
# (8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM).
set -o pipefail
G=${GCTR:-decode}
OUT=gpurun_out/gctr_$G
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $OUT/p*
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
            "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE" \
            "TCP_TCC_READ_REQ_LATENCY TCP_TCP_LATENCY TCP_UTCL1_TRANSLATION_MISS TCP_READ_TAGCONFLICT_STALL_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_BUFFER_COALESCED_READ_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_LDS"; do
  i=$((i + 1))
  GCTR=$G timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python bench/gemm_counters.py > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($pass) rc=$rc"; tail -5 $OUT/p$i.log; [ $rc -eq 137 ] && exit 1; fi
done
python scripts/gemm_counter_summary.py $OUT > $OUT/summary.md
cat $OUT/summary.md
