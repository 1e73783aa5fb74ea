#!/bin/bash
# Round 4: gemm_pf (coalesced epilogue) and gemm_rw (natural k order) numerics + benches.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step() {   # step <log> <limit> <command...>: a failing step is reported, a crash / time limit ends the call
  local log=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/$log 2>&1
  local rc=$?
  tail -${TAILN:-3} gpurun_out/$log
  case $rc in
    0) ;;
    124|137|134|139) echo "STOP: $log rc=$rc"; exit $rc ;;
    *) echo "FAILED: $log rc=$rc" ;;
  esac
}
step r4c_pf_tests.log 300 $T tests/test_gemm_gpu.py -k "pf_"
TAILN=40 step r4c_pf_bench.log 300 python -u bench/pp_bench.py --no-decode --prefill 32768 8192 --rounds 2
step r4c_rw_tests.log 400 $T tests/test_gemm_rw_gpu.py
TAILN=60 step r4c_rw_bench.log 300 python -u bench/rw_bench.py --rounds 3 --ns 3 4 5
