# Round 5: larger decode batches after the medium-M dispatch fix (M = 384 / 512 decode GEMMs used
# gemm_pf before), and the 70B / Mixtral B=256 rows of the README table
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/r5y.txt
for args in "--batch 384" "--batch 512" "--batch 128" "--batch 64"; do
  $T 400 python bench.py $args --steps 3 --warmup 1 > gpurun_out/r5y.log 2>&1 || { echo "bench $args failed"; tail -20 gpurun_out/r5y.log; exit 1; }
  echo "[$args] $(tail -1 gpurun_out/r5y.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], "ttft", r["ttft_p50_ms"], "itl", r["itl_p50_ms"])')" | tee -a gpurun_out/r5y.txt
done
$T 600 python bench.py --model llama3-70b --batch 256 --steps 1 --warmup 1 > gpurun_out/r5y.log 2>&1 || { echo "70b failed"; tail -20 gpurun_out/r5y.log; exit 1; }
echo "[70b 256] $(tail -1 gpurun_out/r5y.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], "ttft", r["ttft_p50_ms"], "itl", r["itl_p50_ms"])')" | tee -a gpurun_out/r5y.txt
