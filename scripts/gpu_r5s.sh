# Round 5: persistent MoE prefill with the static tile walk (gemm_pf MOE mode bit 1) vs gemm_pp_moe
# vs the dynamic queue: MoE GPU tests, then Mixtral B=256 interleaved
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_moe_gpu.py \
  > gpurun_out/r5s_tests.log 2>&1 || { grep -E "^FAILED|passed|failed" gpurun_out/r5s_tests.log | tail; exit 1; }
grep -E "passed|failed" gpurun_out/r5s_tests.log | tail -2
: > gpurun_out/r5s_mixtral.txt
for i in 1 2; do
  for kn in "moe_persistent=0" "moe_persistent=1" "moe_persistent=1,pf_dynamic=on"; do
    DLLM_KNOBS="$kn" $T 400 python bench.py --model mixtral-8x7b --steps 2 --warmup 1 > gpurun_out/r5s_mixtral.log 2>&1 || { echo "mixtral [$kn] failed"; tail -30 gpurun_out/r5s_mixtral.log; exit 1; }
    echo "mixtral [$kn]: $(tail -1 gpurun_out/r5s_mixtral.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], "ttft", r["ttft_p50_ms"], "itl", r["itl_p50_ms"])')" | tee -a gpurun_out/r5s_mixtral.txt
  done
done
