# Round 5 baseline: default bench + origin of the torch kernels in a serving round.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r5a_bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/r5a_bench.log; exit 1; }
tail -1 gpurun_out/r5a_bench.log
timeout -k 10 400 python bench/debug/torch_op_origins.py > gpurun_out/r5a_origins.log 2>&1 || { echo "origins failed"; tail -40 gpurun_out/r5a_origins.log; exit 1; }
head -60 gpurun_out/r5a_origins.log
