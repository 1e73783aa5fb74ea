#!/bin/bash
# Llama-3-70B decode down on split gemm_pp 128-column tiles (nt) vs gemm_wide: numerics, then bench A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
DLLM_KNOBS="pp_down_min_k=16384" $T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wide or large_m or medium or swiglu or long_k" \
  > gpurun_out/r6ab_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6ab_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6ab_tests.txt | head -20; exit $rc; }
: > gpurun_out/r6ab_bench.jsonl
for cfg in dn base dn base; do
  K=""; [ $cfg = dn ] && K="pp_down_min_k=16384"
  DLLM_KNOBS="$K" $T 400 python -u bench.py --model llama3-70b --steps 2 --warmup 1 > gpurun_out/r6ab_bench_$cfg.log 2>&1 \
    || { tail -n 30 gpurun_out/r6ab_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/r6ab_bench_$cfg.log | sed "s/^/$cfg /" >> gpurun_out/r6ab_bench.jsonl
  echo "$cfg $(grep -o '"value": [0-9.]*\|"itl_p50_ms": [0-9.]*\|"ttft_p50_ms": [0-9.]*' gpurun_out/r6ab_bench_$cfg.log | tr '\n' ' ')"
done
