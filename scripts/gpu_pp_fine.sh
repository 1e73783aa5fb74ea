# Sub-layer pipeline cuts: GPU tests, 1-GPU bench, per-stage decode times of the half-layer vs
# sub-layer plans (bench/pp_stage_times.py), and the multi-process IPC rehearsal on the new plans.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -2 gpurun_out/tests_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 900 python -u bench/pp_stage_times.py ${STAGE_ARGS:-} > gpurun_out/pp_stage_times.log 2>&1 || { echo "stage times failed"; tail -40 gpurun_out/pp_stage_times.log; exit 1; }
cat gpurun_out/pp_stage_times.log
PP_N="${PP_N:-2 4}" PP_TRANSPORT=ipc PP_BATCH=256 bash scripts/gpu_pp_rehearsal.sh
