# Round 5: did gemm_pf's static walk regress this round?  Same box, interleaved: the round-4 tree's
# kernels (_r4tree, built from commit 54efb80) vs the current ones, prefill projections at T = 32768
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/r5r_ab.txt
for i in 1 2; do
  (cd _r4tree && $T 300 python bench/pp_bench.py --no-decode --prefill 32768 --rounds 3) > gpurun_out/r5r_r4.txt 2>&1 || { echo "r4 tree failed"; tail -20 gpurun_out/r5r_r4.txt; exit 1; }
  grep prefill gpurun_out/r5r_r4.txt | sed 's/^/r4  /' | tee -a gpurun_out/r5r_ab.txt
  $T 300 python bench/pp_bench.py --no-decode --prefill 32768 --rounds 3 --pf-variants 16 > gpurun_out/r5r_r5.txt 2>&1 || { echo "r5 tree failed"; tail -20 gpurun_out/r5r_r5.txt; exit 1; }
  grep prefill gpurun_out/r5r_r5.txt | sed 's/^/r5  /' | tee -a gpurun_out/r5r_ab.txt
done
