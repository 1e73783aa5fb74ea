"""Per-rank device-side view of a traced pipeline run (bench.py --trace DIR).

    python scripts/trace_gpu_summary.py DIR

For every rank: the stage's GPU-timed spans (cat "stage": one per microbatch the stage ran, from
the first kernel it enqueued to the last, so a span also contains device waits on its input hop)
by kind -- count, mean, p50, p90 -- and the device idle time between consecutive spans."""
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main(d):
    for path in sorted(glob.glob(os.path.join(d, "trace_rank*.json"))):
        evs = [e for e in json.load(open(path))["traceEvents"] if e.get("ph") == "X" and e.get("cat") == "stage"]
        evs.sort(key=lambda e: e["ts"])
        by = defaultdict(list)
        for e in evs:
            by[e["name"]].append(e["dur"])
        gaps = [max(0.0, b["ts"] - (a["ts"] + a["dur"])) for a, b in zip(evs, evs[1:])]
        rank = os.path.basename(path)[len("trace_rank"):-len(".json")]
        parts = [f"{k} n={len(v)} mean={statistics.mean(v) / 1e3:.2f}ms p50={statistics.median(v) / 1e3:.2f}ms "
                 f"p90={sorted(v)[int(0.9 * (len(v) - 1))] / 1e3:.2f}ms" for k, v in sorted(by.items())]
        if gaps:
            parts.append(f"gaps sum={sum(gaps) / 1e3:.1f}ms p50={statistics.median(gaps) / 1e3:.3f}ms "
                         f"max={max(gaps) / 1e3:.1f}ms")
        print(f"rank {rank}: " + " | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
