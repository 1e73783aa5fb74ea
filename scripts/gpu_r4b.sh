#!/bin/bash
# Round 4, second GPU pass: per-kernel decode trace of bench.py with the register-weight GEMMs
# (PROF_KNOBS), then the production-shape correctness test with its achieved errors recorded.
set -o pipefail
mkdir -p gpurun_out
TRACE_TAG=${TRACE_TAG:-rw_b256} DLLM_KNOBS="${PROF_KNOBS:-rw=all}" bash scripts/gpu_trace.sh || exit 1
rm -f gpurun_out/production_shape_errors.jsonl
DLLM_KNOBS="${PROF_KNOBS:-rw=all}" timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread tests/test_production_shapes_gpu.py \
  > gpurun_out/r4b_prod.log 2>&1 || { tail -40 gpurun_out/r4b_prod.log; exit 1; }
tail -3 gpurun_out/r4b_prod.log
