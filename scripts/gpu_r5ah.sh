# Round 5: pp2 stand-in slow mode -- traced runs (per-stage GPU spans and host spans)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1
: > gpurun_out/r5ah.txt
for i in 1 2 3; do
  rm -rf gpurun_out/r5ah_tr$i
  DLLM_TRANSPORT=rccl $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
    --hang-dump 90 --comm-timeout 120 --trace gpurun_out/r5ah_tr$i > gpurun_out/r5ah_pp.log 2>&1 || { grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5ah_pp.log | tail -30; exit 1; }
  { echo "run $i: $(grep '^{' gpurun_out/r5ah_pp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("stage_busy_frac"), "itl", r.get("itl_p50_ms"), "ttft", r.get("ttft_p50_ms"))')";
    python scripts/trace_gpu_summary.py gpurun_out/r5ah_tr$i; python scripts/trace_host_summary.py gpurun_out/r5ah_tr$i; } | tee -a gpurun_out/r5ah.txt
done
