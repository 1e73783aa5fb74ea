#!/bin/bash
# Counters: prefill attention v7 vs the persistent v9 at 32 x 1k / 8 x 4k / 1 x 16k (rope form).
set -o pipefail
OUT=gpurun_out/actr6p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf $OUT/p*
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d $OUT/p$i -o run --output-format csv -- python bench/prefill_attn_bench.py --rope --versions 7 9 --shapes 32x1024 8x4096 1x16384 --reps 3 > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($pass) rc=$rc"; tail -5 $OUT/p$i.log; [ $rc -eq 137 ] && exit 1; fi
done
python scripts/gemm_counter_summary.py $OUT > $OUT/summary.md
cp $OUT/summary.md gpurun_out/r6p_attn_counters.md; cat $OUT/summary.md
# the whole GPU suite on the tree
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r6p_tests.txt 2>&1
rc=$?
tail -n 3 gpurun_out/r6p_tests.txt
exit $rc
