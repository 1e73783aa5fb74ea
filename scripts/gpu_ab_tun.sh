set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for t in old new; do
    f=$GRAFT_REPO_ROOT/distributed_llms_amd/tuning/tunableop_gfx950.csv; [ $t = old ] && f=$GRAFT_REPO_ROOT/build/tun_old.csv
    DLLM_TUNABLEOP_FILE=$f timeout -k 10 600 python bench.py > gpurun_out/abt_${t}_$i.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/abt_${t}_$i.log; exit 1; }
    echo "table=$t run $i: $(tail -1 gpurun_out/abt_${t}_$i.log | cut -c80-200)"
  done
done
