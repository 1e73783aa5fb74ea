#!/bin/bash
# decode qkv / o / down: gemm_pp 128-column tiles with K splits filling the CUs, vs today's gemm_wide.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/debug/medium_m_sweep.py --m 256 --no-wide --shapes qkv o down \
  --pp 128:4 128:5 128:6 128:8 128:8:nt 128:10 128:16 > gpurun_out/r6w_decode_pp_split.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6w_decode_pp_split.txt
exit $rc
