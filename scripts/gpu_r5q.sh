# Round 5: rocprofv3 kernel traces of the B=256 bench (Llama-3-8B, Mixtral) on the final dispatch
set -o pipefail
TRACE_TAG=r5_b256 bash scripts/gpu_trace.sh && TRACE_TAG=r5_mixtral_b256 PROF_ARGS="--model mixtral-8x7b" bash scripts/gpu_trace.sh
