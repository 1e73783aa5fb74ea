# gate|up (SwiGLU) wide GEMM at decode M: default (one 256-row tile, 224 WGs) vs a 128-row tile
# override (448 WGs) vs a 2-way K split (448 WGs + SwiGLU split-K reduce). Cold rotating weights.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py --wide --m 128 192 256 384 --shapes gate_up_8b --variants 32769 49153 > gpurun_out/gateup_ab_s1.log 2>&1 || { echo "s1 failed"; tail -30 gpurun_out/gateup_ab_s1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gateup_ab_s1.log
timeout -k 10 300 python bench/gemm_bench.py --wide --splits 2 --m 128 192 256 384 --shapes gate_up_8b --variants 32769 > gpurun_out/gateup_ab_s2.log 2>&1 || { echo "s2 failed"; tail -30 gpurun_out/gateup_ab_s2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gateup_ab_s2.log
