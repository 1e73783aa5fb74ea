# In-engine A/B of kernel-dispatch knobs (distributed_llms_amd/knobs.py):
#   AB_RUNS="base: v1:wide_variant=1 noq:defer_qkv=1;defer_o=0" AB_ARGS="--batch 256" bash scripts/gpu_ab_knobs.sh
# each run: bench.py with DLLM_KNOBS set to the spec after the colon (';' separates knobs).
set -o pipefail
mkdir -p gpurun_out
for spec in $AB_RUNS; do
  name=${spec%%:*}; kn=${spec#*:}; kn=${kn//;/,}
  DLLM_KNOBS="$kn" timeout -k 10 400 python bench.py --steps 2 --warmup 1 ${AB_ARGS:-} > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }
  echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d.get("kernel_knobs"))')"
done
