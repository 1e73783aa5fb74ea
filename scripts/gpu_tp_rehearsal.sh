# Tensor-parallel rehearsal on a 1-GPU box: torchrun tp2 ranks both on cuda:0, collectives over
# gloo (RCCL refuses two ranks on one device).  Exercises the TP forward (local heads, sharded
# GEMMs, vocab-parallel argmax) on the GPU kernels and the leader/follower step broadcast.
set -o pipefail
mkdir -p gpurun_out
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --parallelism tp --batch ${TP_BATCH:-16} --gen-len 32 --steps 1 --warmup 1 > gpurun_out/tp_rehearsal_2.log 2>&1 || { echo "tp2 rehearsal failed"; tail -40 gpurun_out/tp_rehearsal_2.log; exit 1; }
grep '^{' gpurun_out/tp_rehearsal_2.log | cut -c1-600
# pp2 x tp2: four ranks on cuda:0 (lanes: activations + ids ring per TP rank)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --parallelism pp --tp 2 --batch ${TP_BATCH:-16} --gen-len 32 --steps 1 --warmup 1 > gpurun_out/pptp_rehearsal_4.log 2>&1 || { echo "pp2xtp2 rehearsal failed"; tail -40 gpurun_out/pptp_rehearsal_4.log; exit 1; }
grep '^{' gpurun_out/pptp_rehearsal_4.log | cut -c1-600
