"""Where a gemm_pp prefill launch spends its time, per CU (schedule-2 diagnostic build, variant
bits 64 | 8): every wave records 100 MHz timestamps at kernel entry, main-loop start / end and
after its last output store, plus the CU it ran on.  Per CU the timeline of its workgroups splits
the kernel span into prologue (entry -> loop), loop, epilogue (loop end -> stores done) and idle
gaps between workgroups.

    python bench/pp_timeline.py [--m 8192] [--n 14336] [--k 4096] [--bn 256]
"""
import argparse
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import gemm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192, 32768])
    ap.add_argument("--n", type=int, default=14336)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--bn", type=int, default=256)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    w = (torch.randn(a.n, a.k, device=dev) * 0.02).to(torch.bfloat16)
    var = 64 | 4 | 8 | (1 if a.bn == 128 else 0)
    for m in a.m:
        x = torch.randn(m, a.k, device=dev).to(torch.bfloat16)
        for _ in range(5):
            gemm.linear_pp(x, w, splits=1, variant=var)
        torch.cuda.synchronize()
        grid = (a.n // a.bn) * (-(-m // 256))
        rec = gemm._workspace(dev)[-grid * 512:].view(grid, 4, 128)[:, 0, 8:20].contiguous()
        d = rec.view(torch.float64).cpu()          # [grid, 6]: entry, loop0, loop1, end, hw_id, xcc
        t0 = d[:, 0].min().item()
        span = (d[:, 3].max().item() - t0) / 100.0           # us
        per_cu = defaultdict(list)
        for row in d.tolist():
            per_cu[(int(row[5]), (int(row[4]) >> 8) & 0xFF)].append(row)
        pro, loop, epi, gap, lead, tail = [], [], [], [], [], []
        for wgs in per_cu.values():
            wgs.sort(key=lambda r: r[0])
            lead.append((wgs[0][0] - t0) / 100.0)
            tail.append((d[:, 3].max().item() - wgs[-1][3]) / 100.0)
            for i, r in enumerate(wgs):
                pro.append((r[1] - r[0]) / 100.0)
                loop.append((r[2] - r[1]) / 100.0)
                epi.append((r[3] - r[2]) / 100.0)
                if i + 1 < len(wgs):
                    gap.append((wgs[i + 1][0] - r[3]) / 100.0)
        ncu = len(per_cu)
        tot = lambda xs: sum(xs) / ncu
        fl = 2.0 * m * a.n * a.k
        print(f"M={m} N={a.n} K={a.k} BN={a.bn}: {grid} WGs on {ncu} CUs, span {span:.1f} us "
              f"({fl / span / 1e6:.0f} TF)")
        print(f"  per WG median: prologue {statistics.median(pro):.2f} us, loop {statistics.median(loop):.2f}, "
              f"epilogue {statistics.median(epi):.2f}, gap to the next WG {statistics.median(gap) if gap else 0:.2f}")
        print(f"  per CU mean of the span: prologue {tot(pro):.1f} us, loop {tot(loop):.1f}, epilogue {tot(epi):.1f}, "
              f"gaps {tot(gap):.1f}, start lag {statistics.mean(lead):.1f}, end idle {statistics.mean(tail):.1f}", flush=True)


if __name__ == "__main__":
    main()
