# In-engine A/B of the down-projection wide-kernel cutover (DLLM_WIDE_DOWN_MAX_M) at B = 768 (cap lifted past 512),
# interleaved so box drift hits both settings.
set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 400 env "$@" > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"; }
for b in 768; do
for rep in 1 2; do
for cut in 512 768; do
  run dcut${cut}_b${b}_$rep DLLM_WIDE_DOWN_MAX_M=$cut python bench.py --steps 2 --warmup 1 --batch $b
done
done
done
