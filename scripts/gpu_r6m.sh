#!/bin/bash
# prefill attention v9 (v7 persistent): numerics tests, then v4 / v7 / v9 side by side (two passes).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "prefill" > gpurun_out/r6m_tests.txt 2>&1
rc=$?
tail -n 3 gpurun_out/r6m_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6m_tests.txt | head -20; exit $rc; }
: > gpurun_out/r6m_pattn.txt
for p in 1 2; do
  $T 180 python -u bench/prefill_attn_bench.py --versions 4 7 9 --shapes 256x128 64x512 32x1024 8x4096 2x8192 1x16384 \
    >> gpurun_out/r6m_pattn.txt 2>&1 || { tail -n 20 gpurun_out/r6m_pattn.txt; exit 1; }
done
$T 180 python -u bench/prefill_attn_bench.py --rope --versions 4 7 9 --shapes 256x128 8x4096 1x16384 \
  >> gpurun_out/r6m_pattn.txt 2>&1 || { tail -n 20 gpurun_out/r6m_pattn.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6m_pattn.txt
