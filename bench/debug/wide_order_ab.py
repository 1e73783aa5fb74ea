"""Split-K decode GEMMs in the default vs the K-slice-major workgroup order (knobs.wide_kmajor).

    python bench/debug/wide_order_ab.py [--m 256]

Llama-3-8B / 70B projections through the engine's dispatch (ops.linear), weights rotating through
copies totalling > 1 GB (every call streams its weight from HBM, as a decode step does); arms
interleaved, median us per call.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd import knobs, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256, 128])
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    torch.manual_seed(0)
    shapes = {"qkv_8b": (6144, 4096), "o_8b": (4096, 4096), "down_8b": (4096, 14336),
              "qkv_70b": (10240, 8192), "o_70b": (8192, 8192), "down_70b": (8192, 28672)}
    for m in a.m:
        for name, (n, k) in shapes.items():
            x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            copies = max(2, int((1 << 30) // (n * k * 2)) + 1)
            ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
            it = [0]
            res = {False: [], True: []}
            for r in range(a.rounds):
                for km in (False, True):
                    with knobs.override(wide_kmajor=km):
                        ops.linear(x, ws[0])
                        ev = []
                        for _ in range(10):
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            it[0] += 1
                            e0.record()
                            ops.linear(x, ws[it[0] % copies])
                            e1.record()
                            ev.append((e0, e1))
                        torch.cuda.synchronize()
                        res[km].append(statistics.median(e0.elapsed_time(e1) for e0, e1 in ev) * 1e3)
            d, kmj = statistics.median(res[False]), statistics.median(res[True])
            print(f"M={m:4d} {name:9s} default {d:7.1f} us   kmajor {kmj:7.1f} us   ({100 * (kmj / d - 1):+5.1f} %)",
                  flush=True)
            del ws


if __name__ == "__main__":
    main()
