#!/bin/bash
# Round-end check on the current tree: the whole GPU suite, smoke(), the headline bench, and the
# other single-GPU configs.  A test failure is reported and the benches still run; a crash or a
# time limit ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -4 gpurun_out/final_tests.log
case $rc in 124|137|134|139) echo "STOP tests rc=$rc"; exit $rc ;; 0) ;; *) echo "TESTS FAILED rc=$rc"; grep -E "^FAILED|^ERROR" gpurun_out/final_tests.log | head -20 ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-330
[ -n "${FINAL_MODELS:-}" ] && bash scripts/gpu_models.sh
exit 0
