#!/bin/bash
# medium-M qkv on gemm_wide: numerics, then bench.py --batch 512 A/B (new rule / off / + down on wide at 512).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "medium or large_m or wide" \
  > gpurun_out/r6r_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6r_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6r_tests.txt | head -20; exit $rc; }
: > gpurun_out/r6r_bench.jsonl
for cfg in new off down512 new off down512; do
  case $cfg in
    new) K="" ;;
    off) K="wide_qkv_mid_max_m=0" ;;
    down512) K="wide_down_max_m=512" ;;
  esac
  DLLM_KNOBS="$K" $T 300 python -u bench.py --steps 3 --warmup 1 --batch 512 > gpurun_out/r6r_bench_$cfg.log 2>&1 \
    || { tail -n 30 gpurun_out/r6r_bench_$cfg.log; exit 1; }
  grep '^{' gpurun_out/r6r_bench_$cfg.log | sed "s/^/$cfg /" | tee -a gpurun_out/r6r_bench.jsonl | cut -c1-200
done
