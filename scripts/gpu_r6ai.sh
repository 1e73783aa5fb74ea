#!/bin/bash
# Final rehearsal of the plain multi-rank command on the one GPU (stand-in transport, stage processes
# sharing the device) on the current tree, plus the pipeline GPU tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py tests/test_rccl_standin_gpu.py \
  -m gpu > gpurun_out/r6ai_tests.txt 2>&1
rc=$?
tail -n 2 gpurun_out/r6ai_tests.txt
[ $rc -ne 0 ] && exit $rc
export DLLM_SHARE_GPU=1 DLLM_DATA_BACKEND=gloo DLLM_RCCL_STANDIN=1 DLLM_TRANSPORT=rccl
for n in 2 4; do
  $T 300 python -u bench.py --gpus $n --batch $((512 / n)) --steps 1 --warmup 1 > gpurun_out/r6ai_pp$n.log 2>&1 \
    || { tail -n 30 gpurun_out/r6ai_pp$n.log; exit 1; }
  grep '^{' gpurun_out/r6ai_pp$n.log | grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*\|"transport": "[^"]*"\|"rccl_ranks": [0-9]*\|"parallelism": "[^"]*"' | tr '\n' ' '; echo
done
