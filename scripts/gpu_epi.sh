# LDS-staged GEMM epilogue: bit-exactness tests, then cold microbench (v33 = staged, v9 = no epilogue stores, v17 = no K loop).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "staged or wide_linear or wide_swiglu" > gpurun_out/epi_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
timeout -k 10 300 python bench/gemm_bench.py --wide --m ${EPI_M:-128 256} --shapes qkv_8b o_8b gate_up_8b down_8b lm_head_8b --variants 33 9 17 > gpurun_out/epi_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/epi_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/epi_bench.log
