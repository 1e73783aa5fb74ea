# Round 5: device busy fraction under open-loop load (bench/debug/open_loop_busy.py)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/r5v_busy.txt
for m in 8192 0; do
  timeout -k 10 300 python bench/debug/open_loop_busy.py --rate 176 --mixed $m >> gpurun_out/r5v_busy.txt 2>&1 || { tail -30 gpurun_out/r5v_busy.txt; exit 1; }
done
grep -E "^rate|^steps" gpurun_out/r5v_busy.txt
