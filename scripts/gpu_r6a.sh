#!/bin/bash
# Round 6 start: baseline bench + M = 256 decode projections on gemm_pp split-K vs gemm_wide.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6a_bench.txt 2>&1 || { tail -20 gpurun_out/r6a_bench.txt; exit 1; }
tail -1 gpurun_out/r6a_bench.txt
timeout -k 10 300 python -u bench/debug/decode_pp_split.py > gpurun_out/r6a_split.txt 2>&1 || { tail -20 gpurun_out/r6a_split.txt; exit 1; }
cat gpurun_out/r6a_split.txt
