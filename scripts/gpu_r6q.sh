#!/bin/bash
# medium-M: gemm_wide row tile x K split sweep against today's dispatch.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/debug/medium_m_sweep.py --m 320 384 512 640 768 1024 --bms 128 192 256 \
  > gpurun_out/r6q_sweep.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6q_sweep.txt
exit $rc
