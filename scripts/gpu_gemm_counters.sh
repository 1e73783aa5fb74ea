# Counter passes over bench/gemm_counters.py (kernel trace only, never with sys/runtime traces).
set -o pipefail
mkdir -p gpurun_out/gctr
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/gctr/p*
timeout -k 10 60 rocprofv3 -L > gpurun_out/gctr/list.txt 2>&1 || true
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "TA_TA_BUSY TA_BUSY_avr SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU" "FETCH_SIZE TCC_HIT_sum"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/gctr/p$i -o run --output-format csv -- python bench/gemm_counters.py > gpurun_out/gctr/p$i.log 2>&1 || { echo "pass $i ($pass) failed"; tail -5 gpurun_out/gctr/p$i.log; }
done
python scripts/gemm_counter_summary.py gpurun_out/gctr > gpurun_out/gctr/summary.md
cat gpurun_out/gctr/summary.md
grep -o -E "^[[:space:]]*(TA_[A-Z_]+|SQ_INSTS_[A-Z_]+|SQ_WAIT_[A-Z_]+|TCC_HIT[a-z_]*)" gpurun_out/gctr/list.txt | sort -u | tr -s ' \n' ' ' | head -c 2000; echo
