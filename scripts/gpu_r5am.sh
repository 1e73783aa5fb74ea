#!/bin/bash
# Long prompts in the engine, before (_old/) and after the XCD-aware prefill attention order.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for t in old new; do
    d=.; [ $t = old ] && d=_old
    for cfg in "--batch 32 --prompt-len 2048 --gen-len 32" "--batch 8 --prompt-len 8192 --gen-len 32"; do
      (cd $d && timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 $cfg) > gpurun_out/r5am_run.txt 2>&1 || { tail -20 gpurun_out/r5am_run.txt; exit 1; }
      echo "$t [$cfg] $(tail -1 gpurun_out/r5am_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ')"
    done
  done
done 2>&1 | tee gpurun_out/r5am_long.txt
