#!/bin/bash
# Round 4: gemm_pf schedule variants -- numerics, then the prefill sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "pf_" > gpurun_out/r4h_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4h_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench/pp_bench.py --no-decode --prefill 32768 8192 --shapes qkv o down --rounds 3 --pf-variants 1 2 3 4 5 6 7 > gpurun_out/r4h_bench.log 2>&1 || { tail -20 gpurun_out/r4h_bench.log; exit 1; }
cat gpurun_out/r4h_bench.log
