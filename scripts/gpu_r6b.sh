#!/bin/bash
# Advisor round-5 fixes on the GPU (wide block tables, native comm streams, MoE walk under capture)
# + the gate|up CU-scaling probe.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_engine_gpu.py tests/test_rccl_standin_gpu.py tests/test_rccl_gpu.py tests/test_moe_gpu.py > gpurun_out/r6b_tests.txt 2>&1 || { tail -40 gpurun_out/r6b_tests.txt; exit 1; }
tail -2 gpurun_out/r6b_tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py > gpurun_out/r6b_pipe.txt 2>&1 || { tail -40 gpurun_out/r6b_pipe.txt; exit 1; }
tail -2 gpurun_out/r6b_pipe.txt
timeout -k 10 300 python -u bench/debug/wide_cu_scaling.py > gpurun_out/r6b_cu.txt 2>&1 || { tail -20 gpurun_out/r6b_cu.txt; exit 1; }
cat gpurun_out/r6b_cu.txt
