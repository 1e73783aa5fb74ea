#!/bin/bash
# 70B qkv / o at M = 256: gemm_sq split grids and gemm_wide splits vs today's dispatch.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench/debug/medium_m_sweep.py --m 256 --rounds 3 --shapes qkv70 o70 qkv o \
  --bms 128 256 --splits 2 3 4 5 6 8 --sq 2 4 6 8 16 > gpurun_out/r6ag_70b_proj.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6ag_70b_proj.txt
exit $rc
