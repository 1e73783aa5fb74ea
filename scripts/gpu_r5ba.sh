#!/bin/bash
# Engine A/B (three pairs): swizzled LDS-image epilogue vs the direct-store epilogue (_old/ = 732486d).
set -o pipefail
mkdir -p gpurun_out
for t in old new old new old new; do
  d=.; [ $t = old ] && d=_old
  (cd $d && timeout -k 10 300 python -u bench.py --steps 5 --warmup 1) > gpurun_out/r5ba_run.txt 2>&1 || { tail -20 gpurun_out/r5ba_run.txt; exit 1; }
  echo "$t $(tail -1 gpurun_out/r5ba_run.txt | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"itl_p50_ms": [0-9.]*' | tr '\n' ' ')"
done 2>&1 | tee gpurun_out/r5ba_ab.txt
