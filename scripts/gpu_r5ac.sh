# Round 5: mixed prefill + decode steps through 2-stage GPU pipelines (stand-in and IPC)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v -s --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_mixed_steps" > gpurun_out/r5ac_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|assert" gpurun_out/r5ac_tests.log | tail -8
exit $rc
