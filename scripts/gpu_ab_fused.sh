set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/fr_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fr_tests.log; exit 1; }
tail -1 gpurun_out/fr_tests.log
for i in 1 2; do
  for f in 0 1; do
    DLLM_FUSED_ROPE=$f timeout -k 10 600 python bench.py > gpurun_out/abfr_${f}_$i.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/abfr_${f}_$i.log; exit 1; }
    echo "fused_rope=$f run $i: $(tail -1 gpurun_out/abfr_${f}_$i.log | cut -c80-200)"
  done
done
