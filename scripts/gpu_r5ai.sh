#!/bin/bash
# Grouped V append: numerics, kernel A/B, end-to-end bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rope or prefill" > gpurun_out/r5ai_tests.txt 2>&1 || { tail -30 gpurun_out/r5ai_tests.txt; exit 1; }
tail -3 gpurun_out/r5ai_tests.txt
timeout -k 10 200 python -u bench/rope_bench.py --tokens 32768 --iters 30 > gpurun_out/r5ai_rope.txt 2>&1 && cat gpurun_out/r5ai_rope.txt &&
timeout -k 10 200 python -u bench/rope_bench.py --tokens 4096 --iters 50 >> gpurun_out/r5ai_rope.txt 2>&1 && tail -6 gpurun_out/r5ai_rope.txt &&
for v in 0 1 0 1; do
  DLLM_KNOBS="v_group_append=$v" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r5ai_bench_$v.txt 2>&1 || exit 1
  echo "v_group=$v $(tail -1 gpurun_out/r5ai_bench_$v.txt)"
done
