# A/B: tuned TunableOp table vs library heuristics, Llama-3-8B B=256 (interleaved runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q > gpurun_out/gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
for i in 1 2; do
  for t in 0 1; do
    DLLM_TUNABLEOP=$t timeout -k 10 600 python bench.py > gpurun_out/ab_tun$t_$i.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/ab_tun$t_$i.log; exit 1; }
    echo "tunableop=$t run $i: $(tail -1 gpurun_out/ab_tun$t_$i.log | cut -c1-200)"
  done
done
