#!/bin/bash
# MoE decode expert GEMMs with the LDS-image epilogue: numerics, Mixtral engine A/B vs HEAD (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py tests/test_gemm_gpu.py > gpurun_out/r5ay_tests.txt 2>&1 || { tail -30 gpurun_out/r5ay_tests.txt; exit 1; }
tail -1 gpurun_out/r5ay_tests.txt
for t in old new old new; do
  d=.; [ $t = old ] && d=_old
  (cd $d && timeout -k 10 400 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1) > gpurun_out/r5ay_run.txt 2>&1 || { tail -20 gpurun_out/r5ay_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r5ay_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee gpurun_out/r5ay_mixtral.txt
