"""Summarise rocprofv3 --pmc passes of bench/kernel_counters.py into a per-kernel table.

    python scripts/counters_summary.py gpurun_out/ctr > profiles/kernel_counters.md
"""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    m = re.match(r"_ZN4dllm(\d+)", n)          # mangled template instance: _ZN4dllm<len><name>I...E
    if m:
        ln, rest = int(m.group(1)), n[m.end():]
        targs = re.match(r"I((?:Li\d+E)+)E", rest[ln:])
        args = ",".join(re.findall(r"Li(\d+)E", targs.group(1))) if targs else ""
        return rest[:ln] + (f"<{args}>" if args else "")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    m = re.search(r"dllm::([A-Za-z_0-9]+(?:<[^>]*>)?)", n)
    return m.group(1) if m else n[:40]


def main(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [per dispatch]
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if "dllm" not in r.get("Kernel_Name", ""):
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (d, c), v in per.items():
            vals[names[d]][c].append(v)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "dllm" in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    avg = lambda xs: sum(xs) / len(xs) if xs else float("nan")   # noqa: E731
    print("| kernel | us (median) | LDS bank conflict / LDS active | MFMA util % | wait_any / wave cycles | "
          "FETCH_SIZE KB (x2 = read bytes) | WRITE_SIZE KB | (2*FETCH+WRITE)/time TB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for k in sorted(vals):
        c = vals[k]
        t = sorted(dur.get(k, [float("nan")]))[len(dur.get(k, [0])) // 2]
        lds = avg(c.get("SQ_LDS_BANK_CONFLICT", [])) / max(1.0, avg(c.get("SQ_LDS_IDX_ACTIVE", [1.0])))
        # MFMA_BUSY sums all 1024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs' clocks
        mf = 100 * avg(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])) / max(1.0, avg(c.get("GRBM_GUI_ACTIVE", [1.0])) / 8 * 1024)
        wa = avg(c.get("SQ_WAIT_ANY", [])) / max(1.0, avg(c.get("SQ_WAVE_CYCLES", [1.0])))
        fe, wr = avg(c.get("FETCH_SIZE", [])), avg(c.get("WRITE_SIZE", []))
        bw = (2 * fe + wr) * 1024 / (t * 1e-6) / 1e12 if t == t and t > 0 else float("nan")
        print(f"| `{k}` | {t:.1f} | {lds:.3f} | {mf:.1f} | {wa:.2f} | {fe:.0f} | {wr:.0f} | {bw:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
