#!/bin/bash
# headline knob screen: one bench per knob setting, default at both ends.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
: > gpurun_out/r6u_screen.txt
i=0
for K in "" "attn_target_waves=2048" "attn_target_waves=512" "wide_target_wgs=224" "wide_target_wgs=288" \
         "wide_small_bm=128" "wide_variant=161" "wide_variant_split=129" ""; do
  i=$((i + 1))
  DLLM_KNOBS="$K" timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6u_$i.log 2>&1 \
    || { tail -n 30 gpurun_out/r6u_$i.log; exit 1; }
  echo "[$K] $(grep -o '"value": [0-9.]*\|"itl_p50_ms": [0-9.]*\|"ttft_p50_ms": [0-9.]*' gpurun_out/r6u_$i.log | tr '\n' ' ')" \
    | tee -a gpurun_out/r6u_screen.txt
done
