# Per-row fragment waits in gemm_wide (variant | 32): bit-exactness, cold microbench, in-engine A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "fragment_waits or wide_linear or wide_swiglu" > gpurun_out/sr_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sr_tests.log; exit 1; }
tail -1 gpurun_out/sr_tests.log
timeout -k 10 300 python bench/gemm_bench.py --wide --m ${SR_M:-64 128 256} --shapes qkv_8b o_8b gate_up_8b down_8b lm_head_8b qkv_70b gate_up_70b down_70b --variants 33 > gpurun_out/sr_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/sr_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sr_bench.log
