"""Summarise a rocprofv3 --stats kernel_stats.csv into a markdown table (for profiles/).

    python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [--top 25] [--title ...]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    if n.startswith("_Z"):
        m = re.search(r"dllm\d+([a-z_0-9]+)", n)
        if m:
            n = "dllm::" + m.group(1)
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="")
    ap.add_argument("--per", type=int, default=0, help="divide totals by this (e.g. decode steps)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"## {a.title}\n")
    print(f"total kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")


if __name__ == "__main__":
    main()
