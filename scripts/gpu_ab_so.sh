set -o pipefail
mkdir -p gpurun_out
SO=$(ls distributed_llms_amd/_C_kernels*.so)
for v in ${AB_SO:-plain nt plain nt}; do
  cp altso/$v.so $SO
  timeout -k 10 200 python bench/attn_bench.py --cold --batch 64 256 --ctx 192 1024 > gpurun_out/attn_$v.log 2>&1 || { echo "attn $v failed"; tail -20 gpurun_out/attn_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/attn_$v.log | tail -6
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/ab_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | cut -c1-120
done
