"""What the decode GEMMs' epilogue stores cost: gemm_wide at M = 256 with its stores vs the
no-store ablation (variant bit 8: the K loop and MFMAs run, C / slabs are never written -- timing
only, wrong results).  Weights rotate through > 1 GB of copies (cold, as in a decode step).

    python bench/debug/wide_store_cost.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd.ops import gemm


def main():
    torch.manual_seed(0)
    m = 256
    shapes = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "down": (4096, 14336, False),
              "gate_up": (28672, 4096, True)}
    for name, (n, k, sw) in shapes.items():
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        copies = max(2, int((1 << 30) // (n * k * 2)) + 1)
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        s = gemm.wide_splits(m, n, k, sw)
        it = [0]
        res = {1: [], 9: []}
        for _ in range(7):
            for v in (1, 9):
                ev = []
                for _ in range(10):
                    it[0] += 1
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    gemm.linear_wide(x, ws[it[0] % copies], splits=s, swiglu=sw, variant=v)
                    e1.record()
                    ev.append((e0, e1))
                torch.cuda.synchronize()
                res[v].append(statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3)
        a, b = statistics.median(res[1]), statistics.median(res[9])
        print(f"{name:8s} splits {s}: with stores {a:6.1f} us, no stores {b:6.1f} us ({100 * (a - b) / a:4.1f} % in stores"
              f"{'; both include the split-K reduce' if s > 1 else ''})", flush=True)
        del ws


if __name__ == "__main__":
    main()
