#!/bin/bash
# Llama-3-70B B = 256 kernel trace on the final tree.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TRACE_TAG=r6_70b PROF_BATCH=256 PROF_ARGS="--model llama3-70b" bash scripts/gpu_trace.sh > /dev/null 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace_r6_70b.log; exit 1; }
head -30 gpurun_out/trace_r6_70b.md
