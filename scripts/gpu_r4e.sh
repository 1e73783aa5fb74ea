#!/bin/bash
# Round 4: Mixtral / 70B benches on the current tree (device-side grouped MoE prefill), then the
# Mixtral kernel trace.
set -o pipefail
mkdir -p gpurun_out
for spec in "--model mixtral-8x7b --batch 256" "--model llama3-70b --batch 256"; do
  name=$(echo "$spec" | tr -c 'a-z0-9' '_')
  timeout -k 10 500 python bench.py $spec --steps 2 --warmup 1 > gpurun_out/models_$name.log 2>&1 || { echo "$spec failed"; tail -30 gpurun_out/models_$name.log; exit 1; }
  echo "$spec: $(tail -1 gpurun_out/models_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d.get("ttft_p50_ms"), d.get("itl_p50_ms"))')"
done
TRACE_TAG=mixtral_b256 PROF_ARGS="--model mixtral-8x7b" bash scripts/gpu_trace.sh > /dev/null || exit 1
head -40 gpurun_out/trace_mixtral_b256.md
