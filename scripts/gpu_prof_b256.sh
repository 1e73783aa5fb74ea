# Kernel-level profile of the default Llama-3-8B B=256 bench (rocprofv3 kernel trace + stats).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch ${PROF_BATCH:-256} ${PROF_ARGS:-} > gpurun_out/prof_b256.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_b256.log; exit 1; }
tail -1 gpurun_out/prof_b256.log | cut -c1-300
python scripts/prof_summary.py $(find gpurun_out/prof_b256 -name "*kernel_stats.csv" | head -1) --top 20 --title "B=${PROF_BATCH:-256} ${PROF_ARGS:-}" > gpurun_out/prof_b256.md
cat gpurun_out/prof_b256.md
