# Round 5: re-run the GPU tests that failed in r5o (spinners now in a separate process), the
# production-shape tests (bf16-activation error floor), and the decode GEMMs beside an
# other-process spinner with and without the CU reservation
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_rccl_standin_gpu.py tests/test_production_shapes_gpu.py \
  "tests/test_gemm_gpu.py::test_large_m_uses_hand_written_prefill_gemm" > gpurun_out/r5p_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|gemm_pf solo|static walk|224-workgroup|floor|spinning in" gpurun_out/r5p_tests.log | tail -20
[ $rc -le 1 ] || { echo "tests rc=$rc: stopping"; tail -30 gpurun_out/r5p_tests.log; exit 1; }
$T 300 python scripts/hwq_probe.py gemms > gpurun_out/r5p_gemms.txt 2>&1 || { echo "gemm probe failed"; tail -20 gpurun_out/r5p_gemms.txt; exit 1; }
grep "^gemms" gpurun_out/r5p_gemms.txt
