# A/B of whole kernel-library builds in one GPU session: altso/<name>.so copied over the in-tree
# extension before each run (AB_SO="a b a b"); AB_ATTN=1 adds the cold attention microbench.
set -o pipefail
mkdir -p gpurun_out
SO=$(ls distributed_llms_amd/_C_kernels*.so)
for v in ${AB_SO:-plain nt plain nt}; do
  cp altso/$v.so $SO
  if [ -n "${AB_ATTN:-}" ]; then
    timeout -k 10 200 python bench/attn_bench.py --cold --batch 64 256 --ctx 192 1024 > gpurun_out/attn_$v.log 2>&1 || { echo "attn $v failed"; tail -20 gpurun_out/attn_$v.log; exit 1; }
    echo "== $v"; grep -v amdgpu.ids gpurun_out/attn_$v.log | tail -6
  fi
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 ${AB_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
