#!/bin/bash
# gemm_wide image epilogue with whole-dword, conflict-free image writes: counters test, numerics,
# engine A/B against HEAD (_old/, the half-word image writes).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_counters_gpu.py tests/test_gemm_gpu.py tests/test_engine_gpu.py tests/test_moe_gpu.py > gpurun_out/r5az_tests.txt 2>&1 || { tail -30 gpurun_out/r5az_tests.txt; exit 1; }
tail -1 gpurun_out/r5az_tests.txt
for t in old new old new; do
  d=.; [ $t = old ] && d=_old
  (cd $d && timeout -k 10 300 python -u bench.py --steps 4 --warmup 1) > gpurun_out/r5az_run.txt 2>&1 || { tail -20 gpurun_out/r5az_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r5az_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee gpurun_out/r5az_ab.txt
