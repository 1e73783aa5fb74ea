# gemm_sq at M = 192 / 256 for the unsplit shapes, then in-engine A/B (DLLM_SQ=none vs default).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py --wide --sq --m 192 256 --iters 20 --sq-alt 0 --shapes lm_head_8b gate_up_70b > gpurun_out/sq_bench2.log 2>&1 || { tail -20 gpurun_out/sq_bench2.log; exit 1; }
grep -E "^(lm|gate)" gpurun_out/sq_bench2.log
for arm in none all none all; do
  DLLM_SQ=$arm timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/ab_sq_8b_$arm.log 2>&1 || { tail -20 gpurun_out/ab_sq_8b_$arm.log; exit 1; }
  echo "8b sq=$arm $(grep '^{' gpurun_out/ab_sq_8b_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
for arm in none all; do
  DLLM_SQ=$arm timeout -k 10 600 python bench.py --model llama3-70b --steps 1 --warmup 1 > gpurun_out/ab_sq_70b_$arm.log 2>&1 || { tail -20 gpurun_out/ab_sq_70b_$arm.log; exit 1; }
  echo "70b sq=$arm $(grep '^{' gpurun_out/ab_sq_70b_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
