set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/debug/lm_head_bench.py > gpurun_out/r5ae_head.txt 2>&1 || { tail -20 gpurun_out/r5ae_head.txt; exit 1; }
timeout -k 10 300 python bench/debug/lm_head_bench.py --spinner >> gpurun_out/r5ae_head.txt 2>&1 || { tail -20 gpurun_out/r5ae_head.txt; exit 1; }
grep " us " gpurun_out/r5ae_head.txt
