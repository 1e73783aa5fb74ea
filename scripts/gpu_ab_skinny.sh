set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/sk_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sk_tests.log; exit 1; }
tail -1 gpurun_out/sk_tests.log
for b in 1 8 16 64; do
  for sk in 0 1; do
    DLLM_SKINNY=$sk timeout -k 10 600 python bench.py --batch $b --steps 2 > gpurun_out/absk_${b}_$sk.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/absk_${b}_$sk.log; exit 1; }
    echo "B=$b skinny=$sk: $(tail -1 gpurun_out/absk_${b}_$sk.log | cut -c80-200)"
  done
done
