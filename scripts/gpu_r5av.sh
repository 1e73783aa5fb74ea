#!/bin/bash
# Decode GEMM epilogue store cost (timing ablation).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/debug/wide_store_cost.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5av_store_cost.txt
