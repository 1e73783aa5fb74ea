set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python bench/rope_bench.py > gpurun_out/rope_bench.log 2>&1 || { echo "rope bench failed"; tail -20 gpurun_out/rope_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/rope_bench.log
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/rope_pmc1 -o run --output-format csv -- python bench/rope_bench.py --iters 5 > gpurun_out/rope_pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 gpurun_out/rope_pmc1.log; exit 1; }
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d gpurun_out/rope_pmc2 -o run --output-format csv -- python bench/rope_bench.py --iters 5 > gpurun_out/rope_pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 gpurun_out/rope_pmc2.log; exit 1; }
for f in $(find gpurun_out/rope_pmc1 gpurun_out/rope_pmc2 -name "*counter_collection.csv"); do echo $f; python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "rope" in r.get("Kernel_Name", ""):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, "per dispatch:", [round(x) for x in v[:12]])
PY
done
