#!/bin/bash
# Kernel time summary of the final round-5 tree: rocprofv3 --kernel-trace --stats over the default bench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_final
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python bench.py --steps 2 --warmup 1 > gpurun_out/prof_final.log 2>&1 || { tail -20 gpurun_out/prof_final.log; exit 1; }
tail -1 gpurun_out/prof_final.log | cut -c1-300
find gpurun_out/prof_final -name "*stats*"
