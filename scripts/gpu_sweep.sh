set -o pipefail
mkdir -p gpurun_out
for b in ${SWEEP:-384 512 768}; do
  timeout -k 10 500 python bench.py --steps 2 --warmup 1 --batch $b > gpurun_out/sweep_b$b.log 2>&1 || { echo "bench b=$b failed"; tail -30 gpurun_out/sweep_b$b.log; exit 1; }
  tail -1 gpurun_out/sweep_b$b.log
done
