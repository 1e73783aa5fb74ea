# Round 5: hardware-queue isolation of comm streams and decode GEMMs beside a spinning receive
# (scripts/hwq_probe.py), then the stand-in pipeline tests (exit crash fixed: comm streams are no
# longer destroyed under torch's allocators) and the pp2 rehearsal over the stand-in and over IPC.
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/r5e_hwq.txt
for mode in pool masked_all masked_part priority; do
  $T 60 python scripts/hwq_probe.py queues $mode >> gpurun_out/r5e_hwq.txt 2>&1 || { echo "probe $mode failed"; tail -20 gpurun_out/r5e_hwq.txt; exit 1; }
done
for mode in pool masked_part; do
  GPU_MAX_HW_QUEUES=8 $T 60 python scripts/hwq_probe.py queues $mode >> gpurun_out/r5e_hwq.txt 2>&1 || { echo "probe $mode (8 queues) failed"; tail -20 gpurun_out/r5e_hwq.txt; exit 1; }
done
grep "^queues" gpurun_out/r5e_hwq.txt
$T 180 python scripts/hwq_probe.py gemms > gpurun_out/r5e_gemms.txt 2>&1 || { echo "gemm probe failed"; tail -20 gpurun_out/r5e_gemms.txt; exit 1; }
grep "^gemms" gpurun_out/r5e_gemms.txt
$T 500 python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  "tests/test_pipeline_gpu.py::test_multiprocess_gpu_pipeline_rccl_transport_standin" \
  "tests/test_gemm_gpu.py::test_pf_dispatch_and_graph" \
  "tests/test_rccl_standin_gpu.py::test_gemm_pf_beside_spinning_comm_kernel" \
  > gpurun_out/r5e_tests.log 2>&1
rc=$?
grep -E "^FAILED|passed|failed|static walk|gemm_pf solo" gpurun_out/r5e_tests.log | tail -8
[ $rc -le 1 ] || { echo "tests ended with rc=$rc: stopping"; tail -30 gpurun_out/r5e_tests.log; exit 1; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo
for tr in rccl ipc; do
  if [ $tr = rccl ]; then export DLLM_RCCL_STANDIN=1; else unset DLLM_RCCL_STANDIN; fi
  DLLM_TRANSPORT=$tr $T 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --batch 256 --steps 1 --warmup 1 \
    > gpurun_out/r5e_pp2_${tr}.log 2>&1 || { echo "pp2 $tr failed"; tail -40 gpurun_out/r5e_pp2_${tr}.log; exit 1; }
  echo "pp2 $tr: $(grep '^{' gpurun_out/r5e_pp2_${tr}.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("transport"), r.get("stage_busy_frac"), r.get("itl_p50_ms"))')"
done
