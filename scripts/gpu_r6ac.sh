#!/bin/bash
# 70B gate|up / down at smaller decode M: gemm_pp vs today's dispatch.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench/debug/medium_m_sweep.py --m 64 128 192 224 --no-wide --rounds 3 --shapes gate_up70 down70 gate_up \
  --pp 128:1:nt 256:1:nt 128:4:nt 128:2:nt > gpurun_out/r6ac_70b_small_m.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6ac_70b_small_m.txt
exit $rc
