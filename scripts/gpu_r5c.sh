# Round 5: open-loop latency under Poisson load (mixed prefill + decode steps vs prefill-first) and
# the medium-M GEMM table (257 <= M <= 2048) that sets the gemm_pf cutover.
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r5c_closed.log 2>&1 || { echo "closed-loop bench failed"; tail -30 gpurun_out/r5c_closed.log; exit 1; }
tail -1 gpurun_out/r5c_closed.log | cut -c1-400
: > gpurun_out/r5c_open.jsonl
for spec in "110 8192" "176 8192" "209 8192" "176 512" "209 512" "176 0" "209 0"; do
  set -- $spec
  $T 300 python bench.py --rate $1 --mixed-tokens $2 --steps 5 --warmup 1 > gpurun_out/r5c_open_$1_$2.log 2>&1 || { echo "open loop $spec failed"; tail -30 gpurun_out/r5c_open_$1_$2.log; exit 1; }
  tail -1 gpurun_out/r5c_open_$1_$2.log >> gpurun_out/r5c_open.jsonl
  tail -1 gpurun_out/r5c_open_$1_$2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print("rate", r["offered_rate_rps"], "mixed", r["config"]["mixed_prefill_tokens"], "steps", r["mixed_steps"], "p50", r["p50_latency_ms"], "p99", r["p99_latency_ms"], "ttft50", r.get("ttft_p50_ms"), "ttft99", r.get("ttft_p99_ms"), "itl50", r.get("itl_p50_ms"), "itl99", r.get("itl_p99_ms"), "achieved", r["achieved_rate_rps"])'
done
$T 600 python bench/medium_m_bench.py > gpurun_out/r5c_medium_m.txt 2>&1 || { echo "medium-M bench failed"; tail -30 gpurun_out/r5c_medium_m.txt; exit 1; }
cat gpurun_out/r5c_medium_m.txt
# real RCCL with two ranks on the one device (what the stand-in replaces): record the verdict
$T 180 python scripts/rccl_2rank_probe.py > gpurun_out/rccl_2rank_probe.txt 2>&1; rc=$?
echo "rccl 2-rank probe rc=$rc: $(tail -3 gpurun_out/rccl_2rank_probe.txt)"
