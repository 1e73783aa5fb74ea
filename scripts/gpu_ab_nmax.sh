set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for nm in 0 8192; do
    DLLM_TILED_NMAX=$nm timeout -k 10 600 python bench.py > gpurun_out/ab_nmax${nm}_$i.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/ab_nmax${nm}_$i.log; exit 1; }
    echo "nmax=$nm run $i: $(tail -1 gpurun_out/ab_nmax${nm}_$i.log | cut -c1-160)"
  done
done
