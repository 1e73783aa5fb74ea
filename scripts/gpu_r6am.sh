#!/bin/bash
# 8B down at M = 256: gemm_wide 128-row tiles x K slices vs today's 256-row x 8.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/debug/medium_m_sweep.py --m 256 --rounds 5 --shapes down o \
  --bms 128 256 --splits 2 3 4 5 6 8 > gpurun_out/r6am_down_rows.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6am_down_rows.txt
exit $rc
