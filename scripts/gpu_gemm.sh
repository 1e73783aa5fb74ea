set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gemm_gpu.py -x -q -m gpu > gpurun_out/tg.log 2>&1 || { echo "gemm tests failed"; tail -60 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || { echo "gemm bench failed"; tail -30 gpurun_out/gemm_bench.log; exit 1; }
cat gpurun_out/gemm_bench.log
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/t3.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/b3.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/b3.log; exit 1; }
tail -1 gpurun_out/b3.log
