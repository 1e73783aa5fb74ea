# Session check: GPU tests, smoke, default bench, MoE ring A/B + Mixtral B=256, kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -1 gpurun_out/tests_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench/gemm_bench.py --shapes gate_up_8b gate_up_70b qkv_8b o_8b down_8b --m 256 > gpurun_out/gemm_bench.log 2>&1 || { echo "gemm bench failed"; tail -30 gpurun_out/gemm_bench.log; exit 1; }
cat gpurun_out/gemm_bench.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-600
if [ "${SESSION_MOE:-1}" = "1" ]; then
timeout -k 10 300 python bench/moe_bench.py --tokens 64 128 256 --variants > gpurun_out/moe_bench.log 2>&1 || { echo "moe bench failed"; tail -30 gpurun_out/moe_bench.log; exit 1; }
cat gpurun_out/moe_bench.log
timeout -k 10 600 python bench.py --model mixtral-8x7b --batch 256 --steps 2 --warmup 1 > gpurun_out/bench_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/bench_mixtral.log; exit 1; }
tail -1 gpurun_out/bench_mixtral.log | cut -c1-400
fi
if [ -n "${SESSION_TRACE:-}" ]; then bash scripts/gpu_trace.sh; fi
