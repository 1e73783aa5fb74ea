#!/bin/bash
# prefill attention: staging behind the QK^T MFMAs (v7, v9), one scalar block id per wave, v9's
# double-buffered id lists.  new = the tree, head = the previous commit.  Tests first.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use new
$T 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "prefill" > gpurun_out/r6n_tests.txt 2>&1
rc=$?
tail -n 3 gpurun_out/r6n_tests.txt
[ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/r6n_tests.txt | head -20; exit $rc; }
: > gpurun_out/r6n_pattn.txt
for v in new head new head; do
  use $v
  echo "== $v" >> gpurun_out/r6n_pattn.txt
  $T 180 python -u bench/prefill_attn_bench.py --versions 4 7 9 --shapes 256x128 64x512 32x1024 8x4096 2x8192 1x16384 \
    >> gpurun_out/r6n_pattn.txt 2>&1 || { tail -n 20 gpurun_out/r6n_pattn.txt; exit 1; }
done
use new
grep -v amdgpu.ids gpurun_out/r6n_pattn.txt
