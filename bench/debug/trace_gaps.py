"""GPU idle time between kernels in a rocprofv3 kernel trace (csv), per phase of a serving round.

Decode steps are HIP-graph replays: any host time that is not hidden behind the previous step
shows up as a gap between the last kernel of one step and the first of the next.  This walks the
dispatches in start order (one device), takes the union of busy intervals and reports, for the
decode-attention-delimited steps of the timed region, busy vs idle time and the largest gaps.

    python bench/debug/trace_gaps.py run_kernel_trace.csv [--marker attn_decode_kernel]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="attn_decode_kernel", help="a kernel that runs once per layer per decode step")
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # decode steps: groups of `layers` marker kernels; a step spans from the first kernel after the
    # previous step's last marker's successors ... approximated by marker index boundaries
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    steps = [marks[i: i + a.layers] for i in range(0, len(marks) - a.layers + 1, a.layers)]
    print(f"{len(rows)} dispatches, {len(marks)} '{a.marker}' dispatches, {len(steps)} decode steps")
    if len(steps) < 3:
        return
    # measure from the first marker of step k to the first marker of step k+1
    busy_frac, step_us, idle_us, big = [], [], [], []
    for k in range(len(steps) - 1):
        i0, i1 = steps[k][0], steps[k + 1][0]
        t0, t1 = rows[i0][0], rows[i1][0]
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        for s, e, n in rows[i0:i1]:
            if cur_e is None:
                cur_s, cur_e = s, e
            elif s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        span = t1 - t0
        step_us.append(span / 1e3)
        idle_us.append((span - busy) / 1e3)
        busy_frac.append(busy / span)
        big.extend(gaps)
    print(f"decode step (marker to marker): median {statistics.median(step_us):.1f} us, idle median "
          f"{statistics.median(idle_us):.1f} us ({100 * (1 - statistics.median(busy_frac)):.2f} %)")
    big.sort(reverse=True)
    print("largest gaps (us, next kernel):")
    for g, n in big[:12]:
        print(f"  {g / 1e3:8.1f}  {n[:90]}")
    small = [g for g, _ in big if g < 20_000]
    print(f"gaps < 20 us: {len(small)}, total {sum(small) / 1e3 / max(1, len(steps) - 1):.1f} us per step, "
          f"median {statistics.median(small) / 1e3 if small else 0:.2f} us")


if __name__ == "__main__":
    main()
