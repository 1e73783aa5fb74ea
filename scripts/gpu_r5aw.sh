#!/bin/bash
# gemm_wide epilogue through an LDS image (whole-line stores): numerics, kernel A/B and engine A/B
# against HEAD (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/r5aw_tests.txt 2>&1 || { tail -30 gpurun_out/r5aw_tests.txt; exit 1; }
tail -2 gpurun_out/r5aw_tests.txt
for i in 1 2; do
  echo "== old"; (cd _old && timeout -k 10 200 python -u bench/debug/wide_store_cost.py) || exit 1
  echo "== new"; timeout -k 10 200 python -u bench/debug/wide_store_cost.py || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5aw_ab.txt
for t in old new old new; do
  d=.; [ $t = old ] && d=_old
  (cd $d && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1) > gpurun_out/r5aw_run.txt 2>&1 || { tail -20 gpurun_out/r5aw_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r5aw_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee -a gpurun_out/r5aw_ab.txt
