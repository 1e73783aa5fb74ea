#!/bin/bash
# Open-loop latency on the round-6 tree: 110 / 176 / 209 req/s, mixed steps (budget 8192; 512 at 176).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
: > gpurun_out/r6aj_open.jsonl
for spec in "110 8192" "176 8192" "176 512" "209 8192"; do
  set -- $spec
  $T 300 python -u bench.py --rate $1 --mixed-tokens $2 --steps 5 --warmup 1 > gpurun_out/r6aj_open_$1_$2.log 2>&1 \
    || { tail -30 gpurun_out/r6aj_open_$1_$2.log; exit 1; }
  tail -1 gpurun_out/r6aj_open_$1_$2.log >> gpurun_out/r6aj_open.jsonl
  tail -1 gpurun_out/r6aj_open_$1_$2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print("rate", r["offered_rate_rps"], "mixed", r["config"]["mixed_prefill_tokens"], "steps", r["mixed_steps"], "p50", r["p50_latency_ms"], "p99", r["p99_latency_ms"], "ttft50", r.get("ttft_p50_ms"), "ttft99", r.get("ttft_p99_ms"), "itl50", r.get("itl_p50_ms"), "itl99", r.get("itl_p99_ms"), "achieved", r["achieved_rate_rps"])'
done
