set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/t2.log 2>&1 || { echo "pytest failed rc=$?"; tail -50 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/b2.log 2>&1 || { echo "bench failed rc=$?"; tail -50 gpurun_out/b2.log; exit 1; }
tail -3 gpurun_out/b2.log
