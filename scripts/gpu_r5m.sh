# Round 5: what costs pp2 over the stand-in 24 % (pp4: 3 %)?  The stand-in's CU / LDS footprint
# (channels x LDS per channel) vs the IPC rehearsal on the same box
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
: > gpurun_out/r5m.txt
for kn in "" "standin_lds_kib=0" "standin_channels=1" "standin_lds_kib=0,standin_channels=1" "ipc"; do
  if [ "$kn" = ipc ]; then tr=ipc; unset DLLM_RCCL_STANDIN; k=""; else tr=rccl; export DLLM_RCCL_STANDIN=1; k="$kn"; fi
  DLLM_KNOBS="$k" DLLM_TRANSPORT=$tr $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
    --hang-dump 60 --comm-timeout 120 > gpurun_out/r5m_pp2.log 2>&1 || { echo "pp2 [$kn] failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5m_pp2.log | tail -30; exit 1; }
  echo "pp2 [$tr $kn]: $(grep '^{' gpurun_out/r5m_pp2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"))')" | tee -a gpurun_out/r5m.txt
done
