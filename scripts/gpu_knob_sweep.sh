# In-engine sweep of kernel knobs: bench.py (Llama-3-8B B=256, 2 steps) once per DLLM_KNOBS setting,
# the list run twice, interleaved.  KNOB_SETS: settings separated by ';' ('' = the defaults).
set -o pipefail
mkdir -p gpurun_out
IFS=';' read -r -a SETS <<< "${KNOB_SETS:-;wide_target_wgs=384;wide_small_bm=128;wide_target_wgs=192}"
for pass in 1 2; do
  for k in "${SETS[@]}"; do
    DLLM_KNOBS="$k" timeout -k 10 ${KS_TIMEOUT:-200} python bench.py --steps 2 --warmup 1 ${KS_ARGS:-} > gpurun_out/ks.log 2>&1 || { echo "bench [$k] failed"; tail -20 gpurun_out/ks.log; exit 1; }
    echo "[$k] $(tail -1 gpurun_out/ks.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d.get("kernel_knobs"))')"
  done
done
