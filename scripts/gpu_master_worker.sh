# Master + GPU workers end to end (BASELINE north-star entrypoints) on one MI355X:
#  (1) 1 worker on cuda:0, Llama-3-8B synthetic, 64 requests
#  (2) 2 workers both on cuda:0 (2-stage pipeline, activations host-staged: RCCL refuses
#      two ranks on one device), same workload.
set -o pipefail
mkdir -p gpurun_out
run_case() {  # $1 = name, $2 = workers, $3 = extra env for workers
  local name=$1 nw=$2 port=$((45000 + RANDOM % 10000))
  timeout -k 10 400 python run_master.py --model synthetic:llama3-8b --workers $nw --port $port --auto --bench 64 \
      --prompt-len 128 --gen-len 64 --max-batch 64 --wait-timeout 300 > gpurun_out/mw_${name}_master.log 2>&1 &
  local mpid=$!
  sleep 3
  local wpids=()
  for i in $(seq 1 $nw); do
    env $3 timeout -k 10 380 python run_worker.py --master 127.0.0.1:$port --device cuda:0 --port $((port + i)) \
        > gpurun_out/mw_${name}_worker$i.log 2>&1 &
    wpids+=($!)
  done
  wait $mpid; local rc=$?
  for p in "${wpids[@]}"; do kill $p 2>/dev/null; done
  for p in "${wpids[@]}"; do wait $p 2>/dev/null; done
  echo "[$name] master rc=$rc"; grep -E "tok|metrics|output_tok|latency" gpurun_out/mw_${name}_master.log | tail -4 | cut -c1-400
  return $rc
}
run_case w1 1 "" && run_case w2 2 "DLLM_DATA_BACKEND=gloo"
