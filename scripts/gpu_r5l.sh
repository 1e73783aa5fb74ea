# Round 5: ids receives posted lazily on stage 0's compute stream (in front of their consumer):
# stand-in pipeline tests, then pp2 / pp4 over the stand-in, traced pp2
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  tests/test_rccl_gpu.py > gpurun_out/r5l_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r5l_tests.log | tail -6
[ $rc -eq 0 ] || { echo "tests rc=$rc: stopping"; tail -40 gpurun_out/r5l_tests.log; exit 1; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1
for n in 2 4; do
  DLLM_TRANSPORT=rccl $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29580 + n)) bench.py --gpus $n --batch 256 --steps 1 --warmup 1 \
    --hang-dump 60 --comm-timeout 120 --trace gpurun_out/r5l_tr_pp$n > gpurun_out/r5l_pp$n.log 2>&1 || { echo "pp$n failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5l_pp$n.log | tail -30; exit 1; }
  echo "pp$n stand-in: $(grep '^{' gpurun_out/r5l_pp$n.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("stage_busy_frac"), "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"), r.get("itl_p99_ms"))')"
  python scripts/trace_gpu_summary.py gpurun_out/r5l_tr_pp$n
  python scripts/trace_host_summary.py gpurun_out/r5l_tr_pp$n
done
