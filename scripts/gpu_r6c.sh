#!/bin/bash
# Stream-K gemm_wide: numerics / determinism tests, kernel timings, engine A/B (knobs.wide_streamk).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k streamk > gpurun_out/r6c_tests.txt 2>&1 || { tail -40 gpurun_out/r6c_tests.txt; exit 1; }
tail -3 gpurun_out/r6c_tests.txt
timeout -k 10 300 python -u bench/debug/streamk_bench.py > gpurun_out/r6c_kern.txt 2>&1 || { tail -20 gpurun_out/r6c_kern.txt; exit 1; }
cat gpurun_out/r6c_kern.txt
for t in off on off on; do
  if [ $t = on ]; then export DLLM_KNOBS=wide_streamk=1; else unset DLLM_KNOBS; fi
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6c_run.txt 2>&1 || { tail -20 gpurun_out/r6c_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r6c_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee gpurun_out/r6c_ab.txt
