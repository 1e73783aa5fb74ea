# Round 5: grouped expert prefill GEMMs in isolation (bench/moe_prefill_bench.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/moe_prefill_bench.py > gpurun_out/r5u_moe.txt 2>&1 || { tail -30 gpurun_out/r5u_moe.txt; exit 1; }
grep "T=" gpurun_out/r5u_moe.txt
