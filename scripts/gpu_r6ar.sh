#!/bin/bash
# 70B decode attention with a compile-time 3-slab qkv partial sum (NP = 3) vs the runtime loop: tests, then A/B.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use new
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode" > gpurun_out/r6ar_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6ar_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6ar_tests.txt | head; exit $rc; }
: > gpurun_out/r6ar_bench.jsonl
for v in new old new old; do
  use $v
  $T 400 python -u bench.py --model llama3-70b --steps 2 --warmup 1 > gpurun_out/r6ar_$v.log 2>&1 || { tail -20 gpurun_out/r6ar_$v.log; exit 1; }
  grep '^{' gpurun_out/r6ar_$v.log | sed "s/^/$v /" >> gpurun_out/r6ar_bench.jsonl
  echo "$v $(grep -o '"value": [0-9.]*\|"itl_p50_ms": [0-9.]*' gpurun_out/r6ar_$v.log | tr '\n' ' ')"
done
use new
