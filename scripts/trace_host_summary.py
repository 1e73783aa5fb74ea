"""Per-rank host-side cost of a traced pipeline run (bench.py --trace DIR).

    python scripts/trace_host_summary.py DIR

For every rank: how many decode / prefill microbatches its stage ran, the mean HOST time of one
(span "stage.<kind>", cat "host": building inputs + launching or replaying the graph), the mean
time blocked in the transport spans, and the stall waiting for sampled ids (driver).  At pp = 8 a
stage's GPU time per B = 256 decode microbatch is ~0.8 ms (profiles/pp_stage_balance.md): the host
path per microbatch must stay well under it or the stage becomes host-bound.
"""
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main(d):
    for path in sorted(glob.glob(os.path.join(d, "trace_rank*.json"))):
        evs = json.load(open(path))["traceEvents"]
        spans = defaultdict(list)
        for e in evs:
            if e.get("ph") == "X" and "dur" in e:
                spans[(e.get("cat"), e["name"])].append(e["dur"])
        rank = os.path.basename(path)[len("trace_rank"):-len(".json")]
        parts = []
        for (cat, name), ds in sorted(spans.items()):
            if cat in ("host", "comm"):
                parts.append(f"{name} n={len(ds)} mean={statistics.mean(ds):.0f}us p90={sorted(ds)[int(0.9 * (len(ds) - 1))]:.0f}us")
        print(f"rank {rank}: " + " | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
