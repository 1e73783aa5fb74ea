set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_bench.log
