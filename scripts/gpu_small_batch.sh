set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py --m 1 4 16 64 > gpurun_out/skinny_bench.log 2>&1 || { echo "skinny bench failed"; tail -20 gpurun_out/skinny_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/skinny_bench.log
for b in 1 16; do
  timeout -k 10 600 python bench.py --batch $b --steps 2 > gpurun_out/sb_$b.log 2>&1 || { echo "bench b$b failed"; tail -20 gpurun_out/sb_$b.log; exit 1; }
  echo "B=$b $(tail -1 gpurun_out/sb_$b.log | cut -c1-200)"
done
timeout -k 10 600 python bench.py --model llama3-70b --batch 64 --steps 2 > gpurun_out/sb_70b.log 2>&1 || { echo "70b failed"; tail -20 gpurun_out/sb_70b.log; exit 1; }
echo "70B B=64 $(tail -1 gpurun_out/sb_70b.log | cut -c1-200)"
