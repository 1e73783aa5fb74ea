#!/bin/bash
# Round-6 single-GPU config table on the current tree: 8B at B = 64 / 128 / 384 / 512, Mixtral-8x7B B = 64 / 256,
# Llama-3-70B B = 64.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
: > gpurun_out/r6ah_configs.jsonl
run() {
  tag=$1; shift
  $T 500 python -u bench.py "$@" > gpurun_out/r6ah_$tag.log 2>&1 || { tail -n 20 gpurun_out/r6ah_$tag.log; exit 1; }
  grep '^{' gpurun_out/r6ah_$tag.log | sed "s/^/$tag /" >> gpurun_out/r6ah_configs.jsonl
  echo "$tag $(grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' gpurun_out/r6ah_$tag.log | tr '\n' ' ')"
}
run 8b_b64 --batch 64 --steps 3 --warmup 1
run 8b_b128 --batch 128 --steps 3 --warmup 1
run 8b_b384 --batch 384 --steps 3 --warmup 1
run 8b_b512 --batch 512 --steps 3 --warmup 1
run mix_b64 --model mixtral-8x7b --batch 64 --steps 2 --warmup 1
run mix_b256 --model mixtral-8x7b --batch 256 --steps 2 --warmup 1
run 70b_b64 --model llama3-70b --batch 64 --steps 2 --warmup 1
