#!/bin/bash
# Prefill attention q through an LDS image (whole-line loads): A/B against HEAD (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/r5au_tests.txt 2>&1 || { tail -30 gpurun_out/r5au_tests.txt; exit 1; }
tail -2 gpurun_out/r5au_tests.txt
for i in 1 2; do
  echo "== old"; (cd _old && timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 1x16384 --reps 10) || exit 1
  echo "== new"; timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 1x16384 --reps 10 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5au_prefill_attn.txt
for t in old new old new; do
  d=.; [ $t = old ] && d=_old
  (cd $d && timeout -k 10 300 python -u bench.py --steps 3 --warmup 1) > gpurun_out/r5au_run.txt 2>&1 || { tail -20 gpurun_out/r5au_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r5au_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee -a gpurun_out/r5au_prefill_attn.txt
