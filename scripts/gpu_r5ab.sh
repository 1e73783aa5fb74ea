# Round 5: MoE GPU tests incl. the gemm_pf MOE tile-walk bit-exactness, stand-in tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_moe_gpu.py \
  tests/test_rccl_standin_gpu.py > gpurun_out/r5ab_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|walks" gpurun_out/r5ab_tests.log | tail -8
exit $rc
