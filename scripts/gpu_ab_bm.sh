# A/B of the wide GEMM row-tile override (DLLM_WIDE_SMALL_BM) on the default bench config.
# Round-1 results (B=256, tok/s): base 27,838 / 27,887; o-proj at 128 rows 27,966; qkv+o at 128 26,845;
# qkv+o+down at 128 26,477 -- see profiles/wide_gemm.md.
set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 400 env "$@" > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"; }
for b in ${AB_BATCHES:-256}; do
run base_b$b DLLM_WIDE_SMALL_BM=0 python bench.py --steps 2 --warmup 1 --batch $b
run o128_b$b DLLM_WIDE_SMALL_BM=128 python bench.py --steps 2 --warmup 1 --batch $b
run o64_b$b DLLM_WIDE_SMALL_BM=64 python bench.py --steps 2 --warmup 1 --batch $b
run o192_b$b DLLM_WIDE_SMALL_BM=192 python bench.py --steps 2 --warmup 1 --batch $b
run o128r_b$b DLLM_WIDE_SMALL_BM=128 python bench.py --steps 2 --warmup 1 --batch $b
run base2_b$b DLLM_WIDE_SMALL_BM=0 python bench.py --steps 2 --warmup 1 --batch $b
done
