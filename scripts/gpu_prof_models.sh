set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch 256 > gpurun_out/prof_b256.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_b256.log; exit 1; }
tail -1 gpurun_out/prof_b256.log | cut -c1-300
timeout -k 10 600 python bench.py --model mixtral-8x7b --batch 64 --steps 2 --warmup 1 > gpurun_out/bench_mixtral.log 2>&1 || { echo "mixtral bench failed"; tail -30 gpurun_out/bench_mixtral.log; exit 1; }
tail -1 gpurun_out/bench_mixtral.log
timeout -k 10 600 python bench.py --model llama3-70b --batch 64 --steps 2 --warmup 1 > gpurun_out/bench_70b.log 2>&1 || { echo "70b bench failed"; tail -30 gpurun_out/bench_70b.log; exit 1; }
tail -1 gpurun_out/bench_70b.log
