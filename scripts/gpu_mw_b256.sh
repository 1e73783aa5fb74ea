# Serving path at the bench config: run_master.py + one run_worker.py on cuda:0, Llama-3-8B
# synthetic, 256 requests x (128 prompt, 128 generated), one warmup round, then one timed round.
set -o pipefail
mkdir -p gpurun_out
port=$((45000 + RANDOM % 10000))
timeout -k 10 500 python run_master.py --model synthetic:llama3-8b --workers 1 --port $port --auto --bench ${MW_N:-256} \
    --bench-warmup 1 --prompt-len 128 --gen-len 128 --max-batch ${MW_N:-256} --wait-timeout 300 > gpurun_out/mw256_master.log 2>&1 &
mpid=$!
sleep 3
timeout -k 10 480 python run_worker.py --master 127.0.0.1:$port --device cuda:0 --port $((port + 1)) > gpurun_out/mw256_worker.log 2>&1 &
wpid=$!
wait $mpid; rc=$?
kill $wpid 2>/dev/null; wait $wpid 2>/dev/null
echo "master rc=$rc"; grep -v amdgpu.ids gpurun_out/mw256_master.log | tail -6 | cut -c1-600
exit $rc
