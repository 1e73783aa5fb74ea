# Kernel profiles of Mixtral-8x7B and Llama-3-70B at B=256 (one warmup + one timed round each).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in mixtral-8x7b llama3-70b; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 1 --warmup 1 --batch 256 > gpurun_out/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 gpurun_out/prof_$m.log; exit 1; }
  tail -1 gpurun_out/prof_$m.log | cut -c1-400
  python scripts/prof_summary.py $(find gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1) --top 25 --title "$m B=256" > gpurun_out/prof_$m.md
  cat gpurun_out/prof_$m.md
  rm -rf gpurun_out/prof_$m     # the traces exceed what gpurun copies back; the summary is kept
done
