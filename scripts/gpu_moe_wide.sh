set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/moe_tests.log 2>&1 || { echo "moe tests failed"; tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -1 gpurun_out/moe_tests.log
AB_ARGS="--model mixtral-8x7b --batch ${MB:-256} --steps 2" AB_RUNS="old:DLLM_MOE_WIDE_MIN_PAIRS=0 wide:DLLM_MOE_WIDE_MIN_PAIRS=8" bash scripts/gpu_ab_env.sh
