# Refresh the other single-GPU configs on the current tree (each bench under its own limit).
set -o pipefail
mkdir -p gpurun_out
for spec in "--quant fp8" "--model mixtral-8x7b --batch 256" "--model llama3-70b --batch 256"; do
  name=$(echo "$spec" | tr -c 'a-z0-9' '_')
  timeout -k 10 500 python bench.py $spec --steps 2 --warmup 1 > gpurun_out/models_$name.log 2>&1 || { echo "$spec failed"; tail -30 gpurun_out/models_$name.log; exit 1; }
  echo "$spec: $(tail -1 gpurun_out/models_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["dtype"])')"
done
