#!/bin/bash
# Stream-K diagnostics: steals / waits, the 224-workgroup (one full tile each) and no-partial ablations.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench/debug/streamk_bench.py > gpurun_out/r6d_kern.txt 2>&1 || { tail -20 gpurun_out/r6d_kern.txt; exit 1; }
cat gpurun_out/r6d_kern.txt
