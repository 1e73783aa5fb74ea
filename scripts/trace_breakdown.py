"""Per-call kernel breakdown from a rocprofv3 kernel-trace CSV, labelled by the kernel that ran
just before on the same queue (so the four decode GEMMs of a layer -- qkv after the norm, o after
attention, gate|up after the norm, down after gate|up -- separate even when they share a template).

    python scripts/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--min-calls 64] [--top 30]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name).replace("void ", "")
    m = re.search(r"dllm::([a-z_0-9]+)(<[^>]*>)?", n)
    if m:
        return "dllm::" + m.group(1) + (m.group(2) or "")
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--min-calls", type=int, default=64)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    prev = "start"
    for r in rows:
        k = short(r[name_key])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        per[(k, prev, grid)].append(dur)
        prev = k
    tot = sum(sum(v) for v in per.values())
    print(f"## {a.title}\n\ntotal {tot / 1e3:.1f} ms over {sum(len(v) for v in per.values())} dispatches\n")
    print("| kernel | after | grid | calls | median us | total ms | % |")
    print("|---|---|---|---|---|---|---|")
    items = [(k, v) for k, v in per.items() if len(v) >= a.min_calls]
    items.sort(key=lambda kv: -sum(kv[1]))
    for (k, p, g), v in items[: a.top]:
        print(f"| `{k}` | `{p}` | {g} | {len(v)} | {statistics.median(v):.1f} | {sum(v) / 1e3:.2f} | "
              f"{100 * sum(v) / tot:.1f} |")


if __name__ == "__main__":
    main()
