# Round 5: the whole GPU test suite (no -x: every failure listed)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1140 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5o_gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5o_gpu_tests.log | tail -25
grep -E "bf16-activation floor" gpurun_out/r5o_gpu_tests.log | head
exit $rc
