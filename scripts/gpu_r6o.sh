#!/bin/bash
# prefill attention: v4 / v9 threshold sweep (engine form, q-RoPE in the kernel), then long-prompt
# engine rounds with the auto choice (9) against v7 and v4.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
: > gpurun_out/r6o_pattn.txt
for p in 1 2; do
  $T 180 python -u bench/prefill_attn_bench.py --rope --versions 4 7 9 --shapes 1024x32 512x64 256x128 128x256 96x384 64x512 \
    >> gpurun_out/r6o_pattn.txt 2>&1 || { tail -n 20 gpurun_out/r6o_pattn.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r6o_pattn.txt
: > gpurun_out/r6o_bench.jsonl
for k in 0 7 4 0 7 4; do
  DLLM_KNOBS=prefill_attn=$k $T 300 python -u bench.py --steps 3 --warmup 1 --batch 32 --prompt-len 2048 --gen-len 32 \
    > gpurun_out/r6o_bench_$k.log 2>&1 || { tail -n 30 gpurun_out/r6o_bench_$k.log; exit 1; }
  grep '^{' gpurun_out/r6o_bench_$k.log | sed "s/^/attn=$k /" | tee -a gpurun_out/r6o_bench.jsonl | cut -c1-400
done
