#!/bin/bash
# Counters: the 8B decode gate|up (M = 256) on gemm_pp 128-column tiles vs gemm_wide 256 x 128.
set -o pipefail
OUT=gpurun_out/actr6af
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $OUT/p*
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python bench/debug/medium_m_sweep.py --m 256 --shapes gate_up --pp 128:1:nt --bms 256 --splits 1 --rounds 2 --calls 4 > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($pass) rc=$rc"; tail -5 $OUT/p$i.log; [ $rc -eq 137 ] && exit 1; fi
done
python scripts/gemm_counter_summary.py $OUT > $OUT/summary.md
cp $OUT/summary.md gpurun_out/r6af_gate_up_counters.md; grep -E "gemm_pp|gemm_wide|kernel \|" $OUT/summary.md
