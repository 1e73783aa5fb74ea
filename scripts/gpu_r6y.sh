#!/bin/bash
# Llama-3-70B decode GEMMs (M = 256) and the 8B LM head: gemm_pp 128 / 256-column tiles vs today's dispatch.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench/debug/medium_m_sweep.py --m 256 --no-wide --rounds 3 --shapes qkv70 o70 gate_up70 down70 head \
  --pp 128:1:nt 128:2 128:3 128:4 128:4:nt 256:1:nt 256:2 > gpurun_out/r6y_70b_pp.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6y_70b_pp.txt
exit $rc
