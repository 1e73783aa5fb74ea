set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/fp8_bench.py --m 256 128 --shapes qkv_8b o_8b down_8b gate_up_8b --sweep 1x0 2x0 4x0 8x0 16x0 2x128 4x128 8x128 > gpurun_out/fp8_sweep.log 2>&1 || { tail -30 gpurun_out/fp8_sweep.log; exit 1; }
cat gpurun_out/fp8_sweep.log
