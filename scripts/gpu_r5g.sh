# Round 5: comm streams on high-priority queues + CU reservation for gemm_wide; stand-in GPU tests,
# the pp2 / pp4 rehearsal over the stand-in vs HIP IPC, and the gemm_pf static vs dynamic bench A/B
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_rccl_standin_gpu.py \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_ipc" \
  "tests/test_engine_gpu.py::test_mixed_prefill_decode_steps_gpu" \
  > gpurun_out/r5g_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|static walk|gemm_pf solo|spinning in|224-workgroup" gpurun_out/r5g_tests.log | tail -12
[ $rc -le 1 ] || { echo "tests ended with rc=$rc: stopping"; tail -30 gpurun_out/r5g_tests.log; exit 1; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for n in 2 4; do
  for tr in rccl ipc; do
    if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
    DLLM_TRANSPORT=$tr $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29520 + n)) bench.py --gpus $n --batch 256 --steps 1 --warmup 1 \
      > gpurun_out/r5g_pp${n}_${tr}.log 2>&1 || { echo "pp$n $tr failed"; tail -40 gpurun_out/r5g_pp${n}_${tr}.log; exit 1; }
    echo "pp$n $tr: $(grep '^{' gpurun_out/r5g_pp${n}_${tr}.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("transport"), r.get("stage_busy_frac"), "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"), r.get("itl_p99_ms"))')"
  done
done
unset DLLM_RCCL_STANDIN DLLM_SHARE_GPU DLLM_DATA_BACKEND
for kn in "pf_dynamic=0" "" "pf_dynamic=0" ""; do
  DLLM_KNOBS="$kn" $T 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r5g_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5g_bench.log; exit 1; }
  echo "bench [$kn]: $(tail -1 gpurun_out/r5g_bench.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"))')"
done
