set -o pipefail
mkdir -p gpurun_out
for b in 64 128 256; do
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch $b > gpurun_out/sweep_b$b.log 2>&1 || { echo "bench b=$b failed"; tail -30 gpurun_out/sweep_b$b.log; exit 1; }
  tail -1 gpurun_out/sweep_b$b.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch 128 > gpurun_out/prof2.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof2.log; exit 1; }
echo prof ok
