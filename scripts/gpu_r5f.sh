# Round 5: do high-priority / CU-masked streams get hardware queues of their own (several of them),
# and decode GEMMs beside a spinner that holds LDS (scripts/hwq_probe.py)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/r5f_hwq.txt
for mode in priority_multi masked_multi; do
  $T 60 python scripts/hwq_probe.py queues $mode >> gpurun_out/r5f_hwq.txt 2>&1 || { echo "probe $mode failed"; tail -20 gpurun_out/r5f_hwq.txt; exit 1; }
done
GPU_MAX_HW_QUEUES=8 $T 60 python scripts/hwq_probe.py queues priority_multi >> gpurun_out/r5f_hwq.txt 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r5f_hwq.txt; exit 1; }
grep "^queues" gpurun_out/r5f_hwq.txt
$T 240 python scripts/hwq_probe.py gemms > gpurun_out/r5f_gemms.txt 2>&1 || { echo "gemm probe failed"; tail -20 gpurun_out/r5f_gemms.txt; exit 1; }
grep "^gemms" gpurun_out/r5f_gemms.txt
