#!/bin/bash
# SiLU with the hardware reciprocal (common.h silu_f) A/B on one box: silu = working tree, base = the
# commit before it (ab/_C_kernels_{silu,base}.so, built on the CPU).  GEMM / MoE / SwiGLU GPU tests on
# the silu build, then the prefill gate|up (gemm_pf SwiGLU epilogue) and the decode gate|up
# (gemm_wide SwiGLU) microbenches and the engine bench, interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
SO=distributed_llms_amd/_C_kernels.cpython-310-x86_64-linux-gnu.so
use() { cp ab/_C_kernels_$1.so $SO; }
use silu
$T 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm_gpu.py tests/test_moe_gpu.py \
  tests/test_kernels_gpu.py tests/test_production_shapes_gpu.py > gpurun_out/r6g_tests.txt 2>&1 || { tail -40 gpurun_out/r6g_tests.txt; exit 1; }
tail -3 gpurun_out/r6g_tests.txt
: > gpurun_out/r6g_gemm.txt
: > gpurun_out/r6g_bench.jsonl
for v in silu base silu base; do
  use $v
  echo "== $v" >> gpurun_out/r6g_gemm.txt
  $T 240 python -u bench/pp_bench.py --no-decode --prefill 32768 --shapes gate_up down --rounds 3 >> gpurun_out/r6g_gemm.txt 2>&1 || { tail -20 gpurun_out/r6g_gemm.txt; exit 1; }
  $T 180 python -u bench/debug/wide_cu_scaling.py >> gpurun_out/r6g_gemm.txt 2>&1 || { tail -20 gpurun_out/r6g_gemm.txt; exit 1; }
done
for v in silu base silu base; do
  use $v
  $T 240 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6g_bench_$v.log 2>&1 || { tail -30 gpurun_out/r6g_bench_$v.log; exit 1; }
  grep '^{' gpurun_out/r6g_bench_$v.log | sed "s/^/$v /" | tee -a gpurun_out/r6g_bench.jsonl | cut -c1-200
done
use silu
cat gpurun_out/r6g_gemm.txt
