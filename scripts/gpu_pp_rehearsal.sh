# Multi-process GPU pipeline rehearsal on a 1-GPU box: torchrun pp2/pp4 ranks all on cuda:0,
# control plane and token ring over gloo (RCCL refuses two ranks on one device); activations
# host-staged over gloo, or device to device over HIP IPC with PP_TRANSPORT=ipc. Exercises the
# exact bench.py torchrun path, per-rank stage weights/graphs/KV on the GPU, and the token ring.
set -o pipefail
mkdir -p gpurun_out
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_TRANSPORT=${PP_TRANSPORT:-}
for n in ${PP_N:-2 4}; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --batch ${PP_BATCH:-64} --steps 1 --warmup 1 > gpurun_out/pp_rehearsal_$n.log 2>&1 || { echo "pp$n rehearsal failed"; tail -40 gpurun_out/pp_rehearsal_$n.log; exit 1; }
  grep '^{' gpurun_out/pp_rehearsal_$n.log | cut -c1-600
done
