# Round 5 check: whole GPU suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5x_gpu_tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR|passed|failed" gpurun_out/r5x_gpu_tests.log | tail -12
[ $rc -le 1 ] || { echo "tests rc=$rc: stopping"; tail -30 gpurun_out/r5x_gpu_tests.log; exit 1; }
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5x_smoke.log 2>&1 || { tail -20 gpurun_out/r5x_smoke.log; exit 1; }
tail -1 gpurun_out/r5x_smoke.log
$T 300 python bench.py > gpurun_out/r5x_bench.log 2>&1 || { tail -20 gpurun_out/r5x_bench.log; exit 1; }
tail -1 gpurun_out/r5x_bench.log | cut -c1-500
exit $rc
