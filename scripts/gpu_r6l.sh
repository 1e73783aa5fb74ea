#!/bin/bash
# argmax: four loads in flight per thread + in-thread strict-greater merge.  am = the tree, pre = before.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use am
$T 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k argmax > gpurun_out/r6l_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6l_tests.txt
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/r6l_argmax.txt
: > gpurun_out/r6l_bench.jsonl
for v in am pre am pre; do
  use $v
  echo "== $v" >> gpurun_out/r6l_argmax.txt
  $T 120 python -u bench/debug/argmax_bench.py >> gpurun_out/r6l_argmax.txt 2>&1 || { tail -n 20 gpurun_out/r6l_argmax.txt; exit 1; }
done
for v in am pre am pre; do
  use $v
  $T 240 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6l_bench_$v.log 2>&1 || { tail -n 30 gpurun_out/r6l_bench_$v.log; exit 1; }
  grep '^{' gpurun_out/r6l_bench_$v.log | sed "s/^/$v /" | tee -a gpurun_out/r6l_bench.jsonl | cut -c1-160
done
use am
grep -v amdgpu.ids gpurun_out/r6l_argmax.txt
