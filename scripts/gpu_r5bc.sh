#!/bin/bash
# Prefill attention deferred-max threshold (2^8): numerics, kernel A/B against HEAD (_old/).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_production_shapes_gpu.py > gpurun_out/r5bc_tests.txt 2>&1 || { tail -30 gpurun_out/r5bc_tests.txt; exit 1; }
tail -1 gpurun_out/r5bc_tests.txt
for i in 1 2; do
  echo "== old"; (cd _old && timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 1x16384 --reps 10) || exit 1
  echo "== new"; timeout -k 10 200 python -u bench/prefill_attn_bench.py --rope --versions 4 --shapes 256x128 32x1024 8x4096 1x16384 --reps 10 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5bc_ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
