#!/bin/bash
# Attention softmax / prologue trims, A/B on one box: column max / sum over v_permlane swaps (no
# ds_bpermute), attention.hip built without NaN quieting, the decode new-key patch behind a scalar
# branch, the decode prologue's dependency roots loaded first.  new = the working tree, head = the
# last commit (ab/_C_kernels_{new,head}.so, built on the CPU).  Kernel tests on the new build, then
# the cold decode attention bench, the prefill attention bench (+ the new 32x32x16 kernel, version 6)
# and the engine bench (+ version 6 through DLLM_KNOBS), interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use new
# GPU tests: TESTS (default: the whole suite); the first r6f pass ran everything up to
# test_pipeline_gpu.py (888 passed), so the second runs from there on
# a failing test does not stop the benches; a time limit, abort or crash does (nothing more on the GPU)
$T 900 python -u -m pytest ${PYX--x} -v --timeout 480 --timeout-method thread ${TESTS:-tests} -m gpu \
  > gpurun_out/r6f_tests.txt 2>&1
rc=$?
[ $rc -ne 0 ] && tail -40 gpurun_out/r6f_tests.txt
[ $rc -gt 1 ] && exit $rc
tail -3 gpurun_out/r6f_tests.txt
: > gpurun_out/r6f_attn.txt
: > gpurun_out/r6f_bench.jsonl
: > gpurun_out/r6f_pattn.txt
for v in new head; do
  use $v
  echo "== $v" >> gpurun_out/r6f_attn.txt
  $T 180 python -u bench/attn_bench.py --cold --batch 64 256 --ctx 192 1024 --reps 40 >> gpurun_out/r6f_attn.txt 2>&1 || { tail -20 gpurun_out/r6f_attn.txt; exit 1; }
done
for v in new head new head; do
  use $v
  echo "== $v" >> gpurun_out/r6f_pattn.txt
  V=4; [ $v = new ] && V="4 6 7"
  $T 180 python -u bench/prefill_attn_bench.py --versions $V --shapes 256x128 32x1024 8x4096 1x16384 --reps 10 >> gpurun_out/r6f_pattn.txt 2>&1 || { tail -20 gpurun_out/r6f_pattn.txt; exit 1; }
done
# engine: new (prefill attention v4), head, new with the 32x32 prefill attention (DLLM_KNOBS)
for v in new head new6 new head new6; do
  use ${v%6}
  K=""; [ $v = new6 ] && K="prefill_attn=6"
  DLLM_KNOBS=$K $T 240 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6f_bench_$v.log 2>&1 || { tail -30 gpurun_out/r6f_bench_$v.log; exit 1; }
  grep '^{' gpurun_out/r6f_bench_$v.log | sed "s/^/$v /" | tee -a gpurun_out/r6f_bench.jsonl | cut -c1-200
done
use new
cat gpurun_out/r6f_attn.txt gpurun_out/r6f_pattn.txt
