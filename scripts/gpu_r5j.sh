# Round 5: comm roles back on pool streams (high-priority spinners starved the rehearsal's compute);
# stand-in GPU tests, pp2 / pp4 over the stand-in (default queues and GPU_MAX_HW_QUEUES=8), then the
# gemm_pf static vs dynamic bench A/B
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_rccl_standin_gpu.py \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  > gpurun_out/r5j_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|static walk|gemm_pf solo|spinning in|224-workgroup" gpurun_out/r5j_tests.log | tail -12
[ $rc -le 1 ] || { echo "tests ended with rc=$rc: stopping"; tail -30 gpurun_out/r5j_tests.log; exit 1; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1
for spec in "2 4" "4 4" "2 8" "4 8"; do
  set -- $spec
  GPU_MAX_HW_QUEUES=$2 DLLM_TRANSPORT=rccl $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $((29550 + $1 + $2)) bench.py --gpus $1 --batch 256 --steps 1 --warmup 1 \
    --hang-dump 60 --comm-timeout 120 > gpurun_out/r5j_pp$1_q$2.log 2>&1 || { echo "pp$1 q$2 failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r5j_pp$1_q$2.log | tail -30; exit 1; }
  echo "pp$1 stand-in GPU_MAX_HW_QUEUES=$2: $(grep '^{' gpurun_out/r5j_pp$1_q$2.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("transport"), r.get("stage_busy_frac"), "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"), r.get("itl_p99_ms"))')"
done
unset DLLM_RCCL_STANDIN DLLM_SHARE_GPU DLLM_DATA_BACKEND
for kn in "pf_dynamic=0" "" "pf_dynamic=0" ""; do
  DLLM_KNOBS="$kn" $T 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r5j_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r5j_bench.log; exit 1; }
  echo "bench [$kn]: $(tail -1 gpurun_out/r5j_bench.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], "ttft", r.get("ttft_p50_ms"), "itl", r.get("itl_p50_ms"))')"
done
