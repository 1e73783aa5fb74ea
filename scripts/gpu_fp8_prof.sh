# FP8 mode: numerics tests, engine kernel profile, interleaved bench fp8 / bf16.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1 || { echo "fp8 tests failed"; tail -60 gpurun_out/fp8_tests.log; exit 1; }
tail -1 gpurun_out/fp8_tests.log
PROF_ARGS="--quant fp8" bash scripts/gpu_prof_b256.sh || exit 1
cp gpurun_out/prof_b256.md gpurun_out/prof_b256_fp8.md
for r in 1 2; do for q in fp8 none; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --quant $q > gpurun_out/bench_$q.log 2>&1 || { echo "bench $q failed"; tail -30 gpurun_out/bench_$q.log; exit 1; }
  echo "$q: $(tail -1 gpurun_out/bench_$q.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done; done
