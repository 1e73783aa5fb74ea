# Round 5: pp2 over the stand-in with 32 CUs reserved (both stage processes' spinners) vs 16, vs IPC
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
: > gpurun_out/r5aa_pp.txt
for i in 1 2; do
  for cfg in "rccl comm_reserved_cus=32" "rccl comm_reserved_cus=16" "ipc "; do
    set -- $cfg
    tr=$1; kn=${2:-}
    if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
    DLLM_KNOBS="$kn" DLLM_TRANSPORT=$tr $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
      --hang-dump 90 --comm-timeout 120 > gpurun_out/r5aa_pp.log 2>&1 || { echo "pp2 $cfg failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5aa_pp.log | tail -30; exit 1; }
    echo "pass $i pp2 $tr [$kn]: $(grep '^{' gpurun_out/r5aa_pp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "itl", r.get("itl_p50_ms"))')" | tee -a gpurun_out/r5aa_pp.txt
  done
done
