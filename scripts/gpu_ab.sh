set -o pipefail
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 500 env "$@" > gpurun_out/ab_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/ab_$name.log; exit 1; }; echo "$name: $(tail -1 gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"; }
run auto_b256 DLLM_GEMM=auto python bench.py --steps 2 --warmup 1 --batch 256
run blas_b256 DLLM_GEMM=blas python bench.py --steps 2 --warmup 1 --batch 256
run tiled_b256 DLLM_GEMM=tiled python bench.py --steps 2 --warmup 1 --batch 256
run auto_b512_s2 DLLM_GEMM=auto python bench.py --steps 2 --warmup 1 --batch 512 --streams 2
run auto_b512 DLLM_GEMM=auto python bench.py --steps 2 --warmup 1 --batch 512
