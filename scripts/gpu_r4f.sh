#!/bin/bash
# Round 4: the whole GPU test suite, the headline bench, and its kernel trace (no vendor GEMM
# expected in it).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4f_tests.log
case $rc in 124|137|134|139) echo "STOP tests rc=$rc"; exit $rc ;; 0) ;; *) echo "TESTS FAILED rc=$rc" ;; esac
timeout -k 10 500 python bench.py > gpurun_out/r4f_bench.log 2>&1 || { tail -20 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log | cut -c1-400
TRACE_TAG=r4f_b256 bash scripts/gpu_trace.sh > /dev/null || exit 1
head -32 gpurun_out/trace_r4f_b256.md
