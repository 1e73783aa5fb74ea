# Round 5: open-loop latency after the medium-M dispatch fix (mixed steps at M ~ 300-400 had run on
# gemm_pf), mixed budget 8192 / 512 vs prefill-first, three loads; closed-loop bench as a check
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r5n_closed.log 2>&1 || { echo "closed-loop bench failed"; tail -30 gpurun_out/r5n_closed.log; exit 1; }
tail -1 gpurun_out/r5n_closed.log | cut -c1-300
: > gpurun_out/r5n_open.jsonl
for spec in "110 8192" "110 0" "176 8192" "176 512" "176 0" "209 8192" "209 0"; do
  set -- $spec
  $T 300 python bench.py --rate $1 --mixed-tokens $2 --steps 5 --warmup 1 > gpurun_out/r5n_open_$1_$2.log 2>&1 || { echo "open loop $spec failed"; tail -30 gpurun_out/r5n_open_$1_$2.log; exit 1; }
  tail -1 gpurun_out/r5n_open_$1_$2.log >> gpurun_out/r5n_open.jsonl
  tail -1 gpurun_out/r5n_open_$1_$2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print("rate", r["offered_rate_rps"], "mixed", r["config"]["mixed_prefill_tokens"], "steps", r["mixed_steps"], "p50", r["p50_latency_ms"], "p99", r["p99_latency_ms"], "ttft50", r.get("ttft_p50_ms"), "ttft99", r.get("ttft_p99_ms"), "itl50", r.get("itl_p50_ms"), "itl99", r.get("itl_p99_ms"), "achieved", r["achieved_rate_rps"], "tok/s", r["output_tok_per_s"])'
done
