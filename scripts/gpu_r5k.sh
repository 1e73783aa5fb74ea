# Round 5: why pp2 over the stand-in keeps 76 % of IPC while pp4 keeps 97 % -- traced runs
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for tr in rccl ipc; do
  if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
  DLLM_TRANSPORT=$tr $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
    --hang-dump 60 --trace gpurun_out/r5k_tr_$tr > gpurun_out/r5k_pp2_$tr.log 2>&1 || { echo "pp2 $tr failed"; tail -30 gpurun_out/r5k_pp2_$tr.log; exit 1; }
  echo "pp2 $tr: $(grep '^{' gpurun_out/r5k_pp2_$tr.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "itl", r.get("itl_p50_ms"))')"
  python scripts/trace_gpu_summary.py gpurun_out/r5k_tr_$tr
  python scripts/trace_host_summary.py gpurun_out/r5k_tr_$tr
done
