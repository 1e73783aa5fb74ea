#!/bin/bash
# After the MoE expert GEMM's ordered (deterministic) K-slice reduce and the auto prefill attention
# version: the MoE / engine / pipeline / production-shape GPU tests, then the plain-launch pipeline
# rehearsals of scripts/gpu_r6e.sh part a (8B pp2 / pp4 over the RCCL transport's stand-in).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -v --timeout 480 --timeout-method thread tests/test_moe_gpu.py tests/test_engine_gpu.py \
  tests/test_pipeline_gpu.py tests/test_production_shapes_gpu.py -m gpu > gpurun_out/r6h_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r6h_tests.txt
grep -E "FAILED|rounds agree|round [01]:" gpurun_out/r6h_tests.txt | head -20
[ $rc -gt 1 ] && exit $rc
PART=a SKIP_TESTS=1 bash scripts/gpu_r6e.sh
