# Per-call kernel trace of the default bench (rocprofv3 kernel trace) + role breakdown of the GEMMs.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/trace_${TRACE_TAG:-b256}
rm -rf $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch ${PROF_BATCH:-256} ${PROF_ARGS:-} > $OUT.log 2>&1 || { echo "trace failed"; tail -20 $OUT.log; exit 1; }
tail -1 $OUT.log | cut -c1-300
python scripts/trace_breakdown.py $(find $OUT -name "*kernel_trace.csv" | head -1) --title "B=${PROF_BATCH:-256} ${PROF_ARGS:-}" > $OUT.md
python scripts/prof_summary.py $(find $OUT -name "*kernel_stats.csv" | head -1) --top 25 --title "B=${PROF_BATCH:-256} ${PROF_ARGS:-}" >> $OUT.md
rm -rf $OUT
cat $OUT.md
