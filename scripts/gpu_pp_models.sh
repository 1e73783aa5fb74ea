# Pipeline rehearsal of the big configs on a 1-GPU box: torchrun pp2 ranks sharing cuda:0,
# activations host-staged over gloo (RCCL refuses two ranks on one device).  Exercises the
# Mixtral MoE and Llama-3-70B stage slices through the exact bench.py torchrun path.
set -o pipefail
mkdir -p gpurun_out
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for m in mixtral-8x7b llama3-70b; do
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --model $m --batch ${PP_BATCH:-32} --gen-len 32 --steps 1 --warmup 1 > gpurun_out/pp_$m.log 2>&1 || { echo "pp2 $m failed"; tail -40 gpurun_out/pp_$m.log; exit 1; }
  grep '^{' gpurun_out/pp_$m.log | cut -c1-400
done
