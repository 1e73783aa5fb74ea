# MoE kernels: numerics tests, microbench vs per-expert hipBLASLt, Mixtral end-to-end bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_moe_gpu.py tests/test_gemm_gpu.py -x -q > gpurun_out/moe_tests.log 2>&1 || { echo "moe tests failed"; tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -1 gpurun_out/moe_tests.log
timeout -k 10 300 python bench/moe_bench.py --tokens 16 32 64 128 256 > gpurun_out/moe_bench.log 2>&1 || { echo "moe bench failed"; tail -30 gpurun_out/moe_bench.log; exit 1; }
cat gpurun_out/moe_bench.log
timeout -k 10 600 python bench.py --model mixtral-8x7b --batch 64 --steps 2 --warmup 1 > gpurun_out/bench_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/bench_mixtral.log; exit 1; }
tail -1 gpurun_out/bench_mixtral.log | cut -c1-400
