"""Per-process GPU kernel time from rocprofv3 kernel traces of a multi-process pipeline run.

    python scripts/pp_balance_summary.py DIR [DIR ...]

Each stage process writes its own ``*kernel_trace.csv`` under DIR; the sum of its kernel durations
is that stage's device time over the run (weight-init kernels excluded).  On one GPU the stages
time-share the device, so the absolute sums carry some interference, but max / mean is the
pipeline's stage balance: the slowest stage sets an N-GPU pipeline's rate.  Stage names come
from the kernels only stage 0 (embedding) and the last stage (argmax) run.
"""
import csv
import glob
import os
import sys
from collections import defaultdict

INIT = ("normal", "uniform", "distribution", "randn", "FillFunctor")


def summarize(d):
    per = defaultdict(float)
    names = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                if any(t in k for t in INIT):
                    continue
                pid = row.get("Process_Id") or row.get("Pid") or path
                per[pid] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6   # ms
                if "embedding_kernel" in k:
                    names[pid].add("first")
                if "argmax_kernel" in k:
                    names[pid].add("last")
    if not per:
        print(f"{d}: no kernel traces found")
        return
    rows = sorted(per.items(), key=lambda kv: ("first" not in names[kv[0]], "last" in names[kv[0]], kv[0]))
    mean = sum(per.values()) / len(per)
    print(f"{d}: {len(per)} processes, kernel ms per process (max / mean = {max(per.values()) / mean:.4f})")
    for pid, ms in rows:
        tag = "/".join(sorted(names[pid])) or "mid"
        print(f"  pid {pid:>8s} {tag:10s} {ms:10.1f} ms  ({ms / mean:.3f} x mean)")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        summarize(d)
