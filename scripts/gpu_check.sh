# Full GPU check: pytest -m gpu, smoke(), default bench, short profile. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -2 gpurun_out/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
