set -o pipefail
mkdir -p gpurun_out
for q in fp8 none; do
  timeout -k 10 600 python bench.py --model llama3-70b --steps 1 --warmup 1 --quant $q > gpurun_out/bench_70b_$q.log 2>&1 || { echo "70b $q failed"; tail -30 gpurun_out/bench_70b_$q.log; exit 1; }
  echo "70b $q: $(tail -1 gpurun_out/bench_70b_$q.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["load_s"])')"
done
