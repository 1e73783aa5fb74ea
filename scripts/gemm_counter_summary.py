"""Per-kernel median counters (+ trace durations) from rocprofv3 --pmc pass directories.

    python scripts/gemm_counter_summary.py gpurun_out/gctr
"""
import collections
import csv
import glob
import os
import re
import statistics
import sys


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    m = re.search(r"dllm::([A-Za-z_0-9]+(?:<[^>]*>)?)", n)
    if m:
        return m.group(1)
    m = re.match(r"_ZN4dllm(\d+)", n)
    if m:
        ln, rest = int(m.group(1)), n[m.end():]
        targs = re.findall(r"L[ib](\d+)E", rest[ln:ln + 60])
        return rest[:ln] + ("<" + ",".join(targs) + ">" if targs else "")
    return n[:48]


def main(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per, names = collections.defaultdict(float), {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cols = sorted({c for k in vals.values() for c in k})
    print("| kernel | us | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 2) + "|")
    for k in sorted(vals):
        d = statistics.median(dur[k]) if dur.get(k) else float("nan")
        print(f"| `{k}` | {d:.1f} | " + " | ".join(f"{statistics.median(vals[k][c]):.4g}" if vals[k].get(c) else "-"
                                                  for c in cols) + " |")


if __name__ == "__main__":
    main(sys.argv[1])
