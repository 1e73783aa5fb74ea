# Round 5: pp2 / pp4 over the stand-in, LM head on gemm_sq (default beside comm) vs gemm_pp, interleaved
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1
: > gpurun_out/r5af_pp.txt
for i in 1 2 3; do
  for n in 2 4; do
    for hd in sq pp; do
      DLLM_KNOBS="head_beside_comm=$hd" DLLM_TRANSPORT=rccl $T 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29660 + n)) bench.py --gpus $n --batch 256 \
        --steps 1 --warmup 1 --hang-dump 90 --comm-timeout 120 > gpurun_out/r5af_pp.log 2>&1 || { echo "pp$n $hd failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5af_pp.log | tail -30; exit 1; }
      echo "pass $i pp$n head=$hd: $(grep '^{' gpurun_out/r5af_pp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "itl", r.get("itl_p50_ms"))')" | tee -a gpurun_out/r5af_pp.txt
    done
  done
done
