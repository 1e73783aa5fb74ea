# Round 5: pp8 over the device stand-in and over IPC (eight stage processes on one GPU): the
# lazily posted ids receive, the CU reservation and the comm streams at the deepest pipeline
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for tr in rccl ipc; do
  if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
  DLLM_TRANSPORT=$tr $T 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 8 --batch 128 --steps 1 --warmup 1 \
    --hang-dump 90 --comm-timeout 180 > gpurun_out/r5t_pp8_$tr.log 2>&1 || { echo "pp8 $tr failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5t_pp8_$tr.log | tail -30; exit 1; }
  echo "pp8 $tr: $(grep '^{' gpurun_out/r5t_pp8_$tr.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("transport"), r.get("stage_busy_frac"), "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"))')"
done
