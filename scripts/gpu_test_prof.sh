# GPU tests, then the B=256 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/tests_gpu.log 2>&1 || { echo "GPU tests failed"; tail -60 gpurun_out/tests_gpu.log; exit 1; }
tail -1 gpurun_out/tests_gpu.log
bash scripts/gpu_prof_b256.sh
