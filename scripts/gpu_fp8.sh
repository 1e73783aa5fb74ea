# FP8 W8A8 path: numerics tests, per-shape GEMM bench, in-engine bench vs bf16 (interleaved).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || { echo "fp8 tests failed"; tail -60 gpurun_out/fp8_tests.log; exit 1; }
tail -3 gpurun_out/fp8_tests.log
timeout -k 10 300 python -u bench/fp8_bench.py --m ${FP8_M:-64 128 256 2048} ${FP8_ARGS:-} --out gpurun_out/fp8_gemm.md > gpurun_out/fp8_bench.log 2>&1 || { echo "fp8 bench failed"; tail -30 gpurun_out/fp8_bench.log; exit 1; }
cat gpurun_out/fp8_bench.log
for q in fp8 none; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --quant $q > gpurun_out/bench_$q.log 2>&1 || { echo "bench $q failed"; tail -30 gpurun_out/bench_$q.log; exit 1; }
  echo "$q: $(tail -1 gpurun_out/bench_$q.log | cut -c1-200)"
done
if [ -n "${FP8_MOE:-}" ]; then
  for q in fp8 none; do
    timeout -k 10 500 python bench.py --model mixtral-8x7b --steps 1 --warmup 1 --quant $q > gpurun_out/bench_moe_$q.log 2>&1 || { echo "moe bench $q failed"; tail -30 gpurun_out/bench_moe_$q.log; exit 1; }
    echo "mixtral $q: $(tail -1 gpurun_out/bench_moe_$q.log | cut -c1-220)"
  done
fi
