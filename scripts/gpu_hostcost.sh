# Host-side decode microbatch cost on the GPU box's CPU (the driver's per-microbatch Python/C++ path).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python bench/host_overhead.py --steps 30 > gpurun_out/host_overhead.log 2>&1 || { cat gpurun_out/host_overhead.log; exit 1; }
cat gpurun_out/host_overhead.log
