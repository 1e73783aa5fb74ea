#!/bin/bash
# 8B qkv in 4 K slices vs 5: numerics, then headline A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
DLLM_KNOBS="wide_qkv_splits=4" $T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "wide" \
  > gpurun_out/r6ao_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6ao_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6ao_tests.txt | head -20; exit $rc; }
: > gpurun_out/r6ao_bench.jsonl
for cfg in pp wide pp wide pp wide pp wide; do
  K=""; [ $cfg = pp ] && K="wide_qkv_splits=4"
  DLLM_KNOBS="$K" $T 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6ao_bench_$cfg.log 2>&1 \
    || { tail -n 30 gpurun_out/r6ao_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/r6ao_bench_$cfg.log | sed "s/^/$cfg /" | tee -a gpurun_out/r6ao_bench.jsonl | cut -c1-130
done
grep -o '^[a-z]* \|"itl_p50_ms": [0-9.]*' gpurun_out/r6ao_bench.jsonl | paste - -
