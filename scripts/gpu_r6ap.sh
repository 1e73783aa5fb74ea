#!/bin/bash
# Mixtral-8x7B B = 256 with the o-projection row-tile default (wide_small_bm = 128) vs off.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
: > gpurun_out/r6ap_bench.jsonl
for cfg in new old new old; do
  K=""; [ $cfg = old ] && K="wide_small_bm=0"
  DLLM_KNOBS="$K" $T 400 python -u bench.py --model mixtral-8x7b --batch 256 --steps 2 --warmup 1 > gpurun_out/r6ap_$cfg.log 2>&1 \
    || { tail -n 30 gpurun_out/r6ap_$cfg.log; exit 1; }
  grep '^{' gpurun_out/r6ap_$cfg.log | sed "s/^/$cfg /" >> gpurun_out/r6ap_bench.jsonl
  echo "$cfg $(grep -o '"value": [0-9.]*\|"itl_p50_ms": [0-9.]*' gpurun_out/r6ap_$cfg.log | tr '\n' ' ')"
done
