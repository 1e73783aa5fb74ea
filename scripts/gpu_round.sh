# Full check: GPU tests, smoke, tiled GEMM microbench, default bench, Mixtral bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -1 gpurun_out/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench/gemm_bench.py --tiled --m 128 256 512 --shapes qkv_8b o_8b gate_up_8b down_8b > gpurun_out/tiled_bench.log 2>&1 || { echo "tiled bench failed"; tail -30 gpurun_out/tiled_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tiled_bench.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 600 python bench.py --model mixtral-8x7b --batch 64 --steps 2 --warmup 1 > gpurun_out/bench_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/bench_mixtral.log; exit 1; }
tail -1 gpurun_out/bench_mixtral.log | cut -c1-300
