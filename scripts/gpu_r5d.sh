# Round 5: prefill GEMM schedules (split A / B LDS release, gemm_pf 9-11) vs the shipped one and
# hipBLASLt, then the in-engine A/B of the best, and the Mixtral B=256 bench (persistent MoE prefill).
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python bench/pp_bench.py --no-decode --prefill 32768 8192 --rounds 3 --pf-variants 9 10 11 16 > gpurun_out/r5d_pf_sched.txt 2>&1 || { echo "pf schedule sweep failed"; tail -30 gpurun_out/r5d_pf_sched.txt; exit 1; }
cat gpurun_out/r5d_pf_sched.txt | grep prefill
for kn in "moe_persistent=0" ""; do
  DLLM_KNOBS="$kn" $T 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5d_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/r5d_mixtral.log; exit 1; }
  echo "mixtral [$kn]: $(tail -1 gpurun_out/r5d_mixtral.log | cut -c1-120) ttft $(tail -1 gpurun_out/r5d_mixtral.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ttft_p50_ms"], r["itl_p50_ms"])')"
done
# non-dllm kernels inside one timed Mixtral round (review item 6: ~174 ms of at::native per two rounds in r4)
$T 400 python bench/debug/torch_op_origins.py --model mixtral-8x7b > gpurun_out/r5d_mixtral_origins.txt 2>&1 || { echo "mixtral origins failed"; tail -30 gpurun_out/r5d_mixtral_origins.txt; exit 1; }
tail -25 gpurun_out/r5d_mixtral_origins.txt
