set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_quant_gpu.py -k "splitk or rms or deferred or wide" > gpurun_out/sk_tests.log 2>&1 && tail -3 gpurun_out/sk_tests.log &&
timeout -k 10 120 python bench/splitk_bench.py > gpurun_out/sk_bench.log 2>&1 && timeout -k 10 120 python bench/splitk_bench.py --warm >> gpurun_out/sk_bench.log 2>&1 && cat gpurun_out/sk_bench.log &&
TRACE_TAG=sk bash scripts/gpu_trace.sh > /dev/null 2>&1; grep -n "splitk\|^| \`dllm::gemm_wide" gpurun_out/trace_sk.md | head -20; tail -1 gpurun_out/trace_sk.log | cut -c1-200
