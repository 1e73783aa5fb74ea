# Full check: RCCL transport tests, all GPU tests, smoke, default bench, Mixtral bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_rccl.log 2>&1 || { echo "RCCL tests failed"; tail -60 gpurun_out/tests_rccl.log; exit 1; }
tail -1 gpurun_out/tests_rccl.log
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -1 gpurun_out/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 600 python bench.py --model mixtral-8x7b --batch 64 --steps 2 --warmup 1 > gpurun_out/bench_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/bench_mixtral.log; exit 1; }
tail -1 gpurun_out/bench_mixtral.log | cut -c1-300
