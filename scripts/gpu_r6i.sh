#!/bin/bash
# Prefill attention: version 8 (three phases: QK^T(t) || exp(t-1), P.V(t-1) || max(t)) and the w32
# prologue reorder (first two tiles' DMA before the q loads).  v8 = working tree, new = the r6f build
# (v7 before the prologue change).  Prefill / engine attention GPU tests on v8, then the prefill
# attention bench interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use v8
$T 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "prefill" > gpurun_out/r6i_tests.txt 2>&1
rc=$?
tail -3 gpurun_out/r6i_tests.txt
grep FAILED gpurun_out/r6i_tests.txt | head
[ $rc -gt 1 ] && exit $rc
: > gpurun_out/r6i_pattn.txt
for v in v8 new v8 new; do
  use $v
  echo "== $v" >> gpurun_out/r6i_pattn.txt
  V="4 7"; [ $v = v8 ] && V="4 7 8"
  $T 240 python -u bench/prefill_attn_bench.py --versions $V --shapes 256x128 32x1024 8x4096 1x16384 --reps 10 >> gpurun_out/r6i_pattn.txt 2>&1 || { tail -20 gpurun_out/r6i_pattn.txt; exit 1; }
done
use v8
grep -v amdgpu.ids gpurun_out/r6i_pattn.txt
# Mixtral stage balance again, decode ids now random (bench/pp_stage_times.py decode_batch)
timeout -k 10 300 python -u bench/pp_stage_times.py --model mixtral-8x7b --pp 4 --batch 128 > gpurun_out/r6i_stages_mixtral.txt 2>&1 || { tail -n 30 gpurun_out/r6i_stages_mixtral.txt; exit 1; }
tail -n 6 gpurun_out/r6i_stages_mixtral.txt
