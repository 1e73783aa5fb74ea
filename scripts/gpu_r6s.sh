#!/bin/bash
# decode-M GEMM candidates: gemm_pp (4 waves, 128 x 64 / 128 x 128 wave tiles) against today's dispatch at M = 128 / 256.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench/debug/medium_m_sweep.py --m 128 256 --no-wide \
  --pp 128:1 128:1:nt 128:2 256:1 256:1:nt 256:2 256:4 > gpurun_out/r6s_decode_pp.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/r6s_decode_pp.txt
exit $rc
