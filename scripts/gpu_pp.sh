# gemm_pp: numerics tests, then the decode / prefill microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "pp_" --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { echo "pp tests failed"; tail -40 gpurun_out/pp_tests.log; exit 1; }
tail -2 gpurun_out/pp_tests.log
timeout -k 10 500 python -u bench/pp_bench.py ${PP_ARGS:-} > gpurun_out/pp_bench.log 2>&1 || { echo "pp bench failed"; tail -30 gpurun_out/pp_bench.log; exit 1; }
cat gpurun_out/pp_bench.log
