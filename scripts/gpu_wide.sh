# Wide-M decode GEMM: numerics tests, then cold and warm three-way microbench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k wide > gpurun_out/wide_tests.log 2>&1 || { echo "wide tests failed"; tail -40 gpurun_out/wide_tests.log; exit 1; }
tail -1 gpurun_out/wide_tests.log
for mode in ${WIDE_MODES:-""}; do
timeout -k 10 300 python bench/gemm_bench.py --wide $mode --m 128 256 512 --shapes qkv_8b o_8b gate_up_8b down_8b ${WIDE_ARGS:-} > gpurun_out/wide_bench$mode.log 2>&1 || { echo "wide bench failed"; tail -30 gpurun_out/wide_bench$mode.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wide_bench$mode.log
done
