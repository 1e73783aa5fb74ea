# gemm_gu.hip kernels: numerics, then cold-weight microbench against gemm_wide (decode M = 256).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "gate_up56 or band" --timeout 120 --timeout-method thread > gpurun_out/gu_tests.log 2>&1 || { echo "gu tests failed"; tail -40 gpurun_out/gu_tests.log; exit 1; }
tail -1 gpurun_out/gu_tests.log
timeout -k 10 300 python bench/gemm_bench.py --shapes gate_up_8b qkv_8b o_8b down_8b gate_up_70b --m 256 --gu --band 6 8 > gpurun_out/gu_bench.log 2>&1 || { echo "gu bench failed"; tail -30 gpurun_out/gu_bench.log; exit 1; }
cat gpurun_out/gu_bench.log
