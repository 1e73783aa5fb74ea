# Round 5: decode GEMMs with cold vs cache-resident weights (bench/debug/warm_vs_cold_gemm.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/debug/warm_vs_cold_gemm.py > gpurun_out/r5w_warm.txt 2>&1 || { tail -30 gpurun_out/r5w_warm.txt; exit 1; }
grep "warm/cold" gpurun_out/r5w_warm.txt
