#!/bin/bash
# Prefill attention XCD-aware workgroup order: numerics + A/B against the previous build (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill or rope" > gpurun_out/r5ak_tests.txt 2>&1 || { tail -30 gpurun_out/r5ak_tests.txt; exit 1; }
tail -2 gpurun_out/r5ak_tests.txt
for i in 1 2; do
  echo "== old"; (cd _old && timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 --reps 20) || exit 1
  echo "== new"; timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 --reps 20 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5ak_prefill_attn.txt
