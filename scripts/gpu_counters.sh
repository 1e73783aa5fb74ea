# rocprofv3 hardware counters for every hand-written kernel (separate --pmc passes, kernel trace
# only -- never combined with sys/runtime traces).
set -o pipefail
mkdir -p gpurun_out/ctr
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/ctr/list.txt 2>&1 || true
grep -o -E "SQ_LDS_BANK_CONFLICT|SQ_LDS_IDX_ACTIVE|SQ_VALU_MFMA_BUSY_CYCLES|GRBM_GUI_ACTIVE|SQ_WAIT_ANY|SQ_WAVE_CYCLES|FETCH_SIZE|WRITE_SIZE" gpurun_out/ctr/list.txt | sort -u | tr '\n' ' '; echo
i=0
for pass in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/ctr/p$i -o run --output-format csv -- python bench/kernel_counters.py > gpurun_out/ctr/p$i.log 2>&1 || { echo "pass $i ($pass) failed"; tail -20 gpurun_out/ctr/p$i.log; exit 1; }
done
python scripts/counters_summary.py gpurun_out/ctr > gpurun_out/ctr/summary.md
cat gpurun_out/ctr/summary.md
