# In-engine A/B of the wide-M decode GEMM (DLLM_WIDE) on the default bench config.
set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 400 env "$@" > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"; }
for b in ${AB_BATCHES:-256}; do
for cfg in ${AB_CFGS:-none gate_up gate_up,down all}; do
  w=$cfg; [ "$cfg" = none ] && w=
  run ${cfg//,/+}_b$b DLLM_WIDE=$w python bench.py --steps 2 --warmup 1 --batch $b
done
done
