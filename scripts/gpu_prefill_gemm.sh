set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -x -v -k "grouped or fragment" --timeout 120 --timeout-method thread > gpurun_out/grp_tests.log 2>&1 || { tail -40 gpurun_out/grp_tests.log; exit 1; }
tail -1 gpurun_out/grp_tests.log
timeout -k 10 300 python -u bench/prefill_gemm_bench.py --out gpurun_out/prefill_gemm.md > gpurun_out/prefill_gemm.log 2>&1 || { tail -30 gpurun_out/prefill_gemm.log; exit 1; }
cat gpurun_out/prefill_gemm.log
