# gemm_sq (256 x 256 tile) numerics + microbench against gemm_wide (cold rotating weights).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "sq" --timeout 120 --timeout-method thread > gpurun_out/sq_tests.log 2>&1 || { echo "sq tests failed"; tail -40 gpurun_out/sq_tests.log; exit 1; }
tail -2 gpurun_out/sq_tests.log
timeout -k 10 400 python bench/gemm_bench.py --wide --sq --m ${SQ_M:-192 256} --iters 20 --sq-alt ${SQ_ALT:-0} --shapes ${SQ_SHAPES:-qkv_8b o_8b gate_up_8b down_8b lm_head_8b qkv_70b o_70b gate_up_70b down_70b} > gpurun_out/sq_bench.log 2>&1 || { echo "sq bench failed"; tail -30 gpurun_out/sq_bench.log; exit 1; }
cat gpurun_out/sq_bench.log
