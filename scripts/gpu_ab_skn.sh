# In-engine A/B of the fused split-K + residual + RMSNorm workgroup size (DLLM_SKN_THREADS), B=256,
# plus smoke() (GPU vs CPU fp32 logits) under the 512-thread variant.
set -o pipefail
mkdir -p gpurun_out
DLLM_SKN_THREADS=512 timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/skn_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/skn_smoke.log; exit 1; }
tail -1 gpurun_out/skn_smoke.log
run() { name=$1; shift; timeout -k 10 400 env "$@" > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"; }
for rep in 1 2 3; do
for t in 256 512; do
  run skn${t}_$rep DLLM_SKN_THREADS=$t python bench.py --steps 2 --warmup 1 --batch 256
done
done
