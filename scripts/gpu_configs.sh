# Headline numbers for every single-GPU config.
set -o pipefail
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/cfg_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_$name.log; exit 1; }; echo "$name $(tail -1 gpurun_out/cfg_$name.log | cut -c1-420)"; }
run 8b_b256
run 8b_b512 --batch 512
run 8b_b64 --batch 64
run mixtral_b64 --model mixtral-8x7b --batch 64 --steps 2
run mixtral_b256 --model mixtral-8x7b --batch 256 --steps 2
run 70b_b64 --model llama3-70b --batch 64 --steps 2
run 70b_b256 --model llama3-70b --batch 256 --steps 2
run 8b_b128 --batch 128
