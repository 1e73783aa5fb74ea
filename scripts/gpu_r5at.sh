#!/bin/bash
# Timing ablation (wrong results, no tests): decode attention with K fragments loaded as whole
# 128-byte lines (1 KB contiguous per instruction) vs the shipped half-line pattern (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  echo "== old"; (cd _old && timeout -k 10 200 python -u bench/attn_bench.py --batch 64 256 --ctx 192 1024 4096 --targets 1024 2048) || exit 1
  echo "== ablation"; timeout -k 10 200 python -u bench/attn_bench.py --batch 64 256 --ctx 192 1024 4096 --targets 1024 2048 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5at_attn_kload.txt
