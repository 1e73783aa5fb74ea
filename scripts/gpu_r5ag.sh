# Round 5: probed queue-isolated comm role streams: GPU tests, then pp2 / pp4 over the stand-in x3
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -v -s --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_rccl_standin_gpu.py" "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_mixed_steps" tests/test_rccl_gpu.py > gpurun_out/r5ag_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r5ag_tests.log | tail -6
[ $rc -eq 0 ] || { tail -30 gpurun_out/r5ag_tests.log; exit 1; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
: > gpurun_out/r5ag_pp.txt
for i in 1 2 3; do
  for n in 2 4; do
    for tr in rccl ipc; do
      if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
      DLLM_TRANSPORT=$tr $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29670 + n)) bench.py --gpus $n --batch 256 --steps 1 --warmup 1 \
        --hang-dump 90 --comm-timeout 120 > gpurun_out/r5ag_pp.log 2>&1 || { echo "pp$n $tr failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5ag_pp.log | tail -30; exit 1; }
      echo "pass $i pp$n $tr: $(grep '^{' gpurun_out/r5ag_pp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "itl", r.get("itl_p50_ms"))')" | tee -a gpurun_out/r5ag_pp.txt
    done
  done
done
