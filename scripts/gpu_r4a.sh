#!/bin/bash
# Round 4, first GPU pass: new kernels' numerics, the RCCL transport stand-in on one GPU, then the
# register-weight GEMM bench.  Each step under its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gemm_rw_gpu.py > gpurun_out/r4a_rw_tests.log 2>&1 || { tail -30 gpurun_out/r4a_rw_tests.log; exit 1; }
tail -2 gpurun_out/r4a_rw_tests.log
timeout -k 10 300 python -u bench/rw_bench.py --rounds 3 --ns 3 4 5 > gpurun_out/r4a_rw_bench.log 2>&1 || { tail -30 gpurun_out/r4a_rw_bench.log; exit 1; }
cat gpurun_out/r4a_rw_bench.log
timeout -k 10 400 $T tests/test_moe_gpu.py > gpurun_out/r4a_moe.log 2>&1 || { tail -30 gpurun_out/r4a_moe.log; exit 1; }
tail -2 gpurun_out/r4a_moe.log
timeout -k 10 300 $T tests/test_pipeline_gpu.py -k standin > gpurun_out/r4a_standin.log 2>&1 || { tail -30 gpurun_out/r4a_standin.log; exit 1; }
tail -2 gpurun_out/r4a_standin.log
AB_RUNS="base: rw:rw=all base2: rw2:rw=all" bash scripts/gpu_ab_knobs.sh || exit 1
