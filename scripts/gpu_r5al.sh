#!/bin/bash
# gemm_wide K-slice-major workgroup order: bit-exactness, kernel A/B, in-engine A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wide" > gpurun_out/r5al_tests.txt 2>&1 || { tail -30 gpurun_out/r5al_tests.txt; exit 1; }
tail -2 gpurun_out/r5al_tests.txt
timeout -k 10 400 python -u bench/debug/wide_order_ab.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5al_ab.txt || exit 1
for v in 0 1 0 1; do
  DLLM_KNOBS="wide_kmajor=$v" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r5al_bench_$v.txt 2>&1 || exit 1
  echo "kmajor=$v $(tail -1 gpurun_out/r5al_bench_$v.txt | cut -c1-200) $(tail -1 gpurun_out/r5al_bench_$v.txt | grep -o '"itl_p50_ms": [0-9.]*')"
done
