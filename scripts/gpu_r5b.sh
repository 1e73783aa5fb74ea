# Round 5: device-async RCCL stand-in + gemm_pf dynamic tile queue.
#  1. GPU tests of the stand-in, the gemm_pf queue (beside a spinning kernel), pipelines over it
#  2. pp2 / pp4 rehearsal at B=256 over the stand-in and over HIP IPC (same box)
#  3. bench.py A/B: gemm_pf static vs dynamic tile walk
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 700 python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_rccl_standin_gpu.py \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_ipc" \
  "tests/test_engine_gpu.py::test_mixed_prefill_decode_steps_gpu" \
  tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_moe_gpu.py \
  -k "standin or gemm_pf or pf_ or ipc or mixed or prefill or persistent or queue" \
  > gpurun_out/r5b_tests.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then
  grep -E "^FAILED|^ERROR" gpurun_out/r5b_tests.log | head -20
  # assertion failures (rc 1) still let the measurements run; a timeout, abort or crash ends the call
  [ $rc -eq 1 ] || { echo "tests ended with rc=$rc: stopping"; tail -30 gpurun_out/r5b_tests.log; exit 1; }
fi
grep -E "passed|failed|gemm_pf solo|static walk" gpurun_out/r5b_tests.log | tail -8
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for tr in rccl ipc; do
  for n in 2 4; do
    if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
    DLLM_TRANSPORT=$tr $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --batch 256 --steps 1 --warmup 1 \
      > gpurun_out/r5b_pp${n}_${tr}.log 2>&1 || { echo "pp$n $tr failed"; tail -40 gpurun_out/r5b_pp${n}_${tr}.log; exit 1; }
    echo "pp$n $tr: $(grep '^{' gpurun_out/r5b_pp${n}_${tr}.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("transport"), r.get("stage_busy_frac"))')"
  done
done
unset DLLM_RCCL_STANDIN DLLM_SHARE_GPU DLLM_DATA_BACKEND
for kn in "pf_dynamic=0" "" "pf_dynamic=0" ""; do
  DLLM_KNOBS="$kn" $T 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r5b_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5b_bench.log; exit 1; }
  echo "bench [$kn]: $(tail -1 gpurun_out/r5b_bench.log | cut -c1-200)"
done
