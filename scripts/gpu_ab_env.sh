# Generic in-engine A/B: AB_RUNS="name1:VAR=a,VAR2=b name2:..." -> bench.py tok/s for each (env set per run).
set -o pipefail
mkdir -p gpurun_out
for spec in $AB_RUNS; do
  name=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
  timeout -k 10 400 env $envs python bench.py --steps 2 --warmup 1 ${AB_ARGS:-} > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }
  echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
