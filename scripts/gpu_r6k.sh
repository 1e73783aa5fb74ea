#!/bin/bash
# The whole GPU suite on the committed tree (what the driver runs at round end).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -v --timeout 480 --timeout-method thread tests -m gpu > gpurun_out/r6k_tests.txt 2>&1
rc=$?
tail -n 3 gpurun_out/r6k_tests.txt
grep FAILED gpurun_out/r6k_tests.txt | head -20
exit $rc
