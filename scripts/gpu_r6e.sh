#!/bin/bash
# Round 6 review items 1 and 4 on the one-GPU box:
#  * the plain `python bench.py --gpus N` (self-launched ranks, no torchrun) over the RCCL transport's
#    multi-rank path with the device stand-in, stage processes sharing the GPU;
#  * BASELINE configs 4 / 5 at pipeline depth on the same path: reduced-depth token-exact tests,
#    then full-size Llama-3-70B pp4 / pp8 and Mixtral-8x7B pp4 bench rounds.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
[ "${PART:-a}" = a ] && [ -z "$SKIP_TESTS" ] && { $T 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_pipeline_gpu.py -k "big_model_dims or rccl_transport_standin" > gpurun_out/r6e_tests.txt 2>&1 || { tail -40 gpurun_out/r6e_tests.txt; exit 1; }
tail -6 gpurun_out/r6e_tests.txt; }
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1 DLLM_TRANSPORT=rccl
: > gpurun_out/r6e_bench_${PART:-a}.jsonl
run() {   # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  $T $t python -u bench.py "$@" --comm-timeout 240 > gpurun_out/r6e_$name.log 2>&1 || { echo "$name failed"; grep -v "amdgpu.ids\|Gloo\|socket.cpp" gpurun_out/r6e_$name.log | tail -30; exit 1; }
  grep '^{' gpurun_out/r6e_$name.log | tee -a gpurun_out/r6e_bench_${PART:-a}.jsonl | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print("'$name'", r["value"], r["config"]["parallelism"], r["transport"], "rccl_ranks", r.get("rccl_ranks"), "busy", r.get("stage_busy_frac"), "ranges", r.get("stage_ranges"))'
}
if [ "${PART:-a}" = a ]; then
  run plain_8b_pp2 240 --gpus 2 --batch 256 --steps 1 --warmup 1
  run plain_8b_pp4 240 --gpus 4 --batch 128 --steps 1 --warmup 1
else
  run plain_70b_pp4 420 --gpus 4 --model llama3-70b --batch 64 --steps 1 --warmup 1
  run plain_mixtral_pp4 300 --gpus 4 --model mixtral-8x7b --batch 128 --steps 1 --warmup 1
  run plain_70b_pp8 420 --gpus 8 --model llama3-70b --batch 32 --steps 1 --warmup 1
  unset DLLM_SHARE_GPU DLLM_DATA_BACKEND DLLM_RCCL_STANDIN DLLM_TRANSPORT
  # stage-balance tables: every stage of the plan built and timed one at a time (decode graph replay)
  $T 400 python -u bench/pp_stage_times.py --model llama3-70b --pp 4 8 --batch 64 > gpurun_out/r6e_stages_70b.txt 2>&1 || { tail -30 gpurun_out/r6e_stages_70b.txt; exit 1; }
  $T 300 python -u bench/pp_stage_times.py --model mixtral-8x7b --pp 4 --batch 128 > gpurun_out/r6e_stages_mixtral.txt 2>&1 || { tail -30 gpurun_out/r6e_stages_mixtral.txt; exit 1; }
  tail -n 12 gpurun_out/r6e_stages_70b.txt gpurun_out/r6e_stages_mixtral.txt
fi
