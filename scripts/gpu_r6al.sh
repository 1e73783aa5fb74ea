#!/bin/bash
# Round-6 final check on the committed tree: smoke(), the default bench (the driver's 1-GPU form) and
# the rocprofv3 kernel-trace summary of one bench round (scripts/gpu_trace.sh -> gpurun_out/trace_r6_b256.md).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 900 python -u -m pytest -x --timeout 120 --timeout-method thread tests \
  -q -m gpu > gpurun_out/r6al_tests.txt 2>&1
rc=$?
tail -n 3 gpurun_out/r6al_tests.txt
grep FAILED gpurun_out/r6al_tests.txt | head
[ $rc -gt 1 ] && exit $rc
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6al_smoke.txt 2>&1 || { tail -20 gpurun_out/r6al_smoke.txt; exit 1; }
tail -1 gpurun_out/r6al_smoke.txt
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r6al_bench_$i.log 2>&1 || { tail -20 gpurun_out/r6al_bench_$i.log; exit 1; }
  grep '^{' gpurun_out/r6al_bench_$i.log | cut -c1-400
done
$T 400 python -u bench.py --model llama3-70b --steps 2 --warmup 1 > gpurun_out/r6al_bench_70b.log 2>&1 || { tail -20 gpurun_out/r6al_bench_70b.log; exit 1; }
grep '^{' gpurun_out/r6al_bench_70b.log | cut -c1-200
TRACE_TAG=r6_b256 bash scripts/gpu_trace.sh > /dev/null 2>&1 || { echo "trace failed"; exit 1; }
head -40 gpurun_out/trace_r6_b256.md
