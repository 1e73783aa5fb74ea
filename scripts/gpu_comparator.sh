# HF transformers comparator + Mixtral kernel profile.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench/hf_comparator.py --model llama3-8b --batch 256 > gpurun_out/hf_8b_b256.log 2>&1 || { echo "hf 8b failed"; tail -20 gpurun_out/hf_8b_b256.log; exit 1; }
tail -1 gpurun_out/hf_8b_b256.log
timeout -k 10 600 python bench/hf_comparator.py --model mixtral-8x7b --batch 64 > gpurun_out/hf_mixtral_b64.log 2>&1 || { echo "hf mixtral failed"; tail -20 gpurun_out/hf_mixtral_b64.log; exit 1; }
tail -1 gpurun_out/hf_mixtral_b64.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixtral -o run --output-format csv -- python bench.py --model mixtral-8x7b --batch 64 --steps 1 --warmup 1 > gpurun_out/prof_mixtral.log 2>&1 || { echo "prof mixtral failed"; tail -20 gpurun_out/prof_mixtral.log; exit 1; }
tail -1 gpurun_out/prof_mixtral.log | cut -c1-300
python scripts/prof_summary.py $(find gpurun_out/prof_mixtral -name "*kernel_stats.csv" | head -1) --top 20 --title "Mixtral-8x7B B=64" > gpurun_out/prof_mixtral.md
cat gpurun_out/prof_mixtral.md
