"""Prefill-sized bf16 GEMMs: hipBLASLt (torch, + silu_mul for gate|up) vs the wide kernel with the
grouped row-tile order (gemm_wide variant bit 64, SwiGLU fused into its epilogue).

    python bench/prefill_gemm_bench.py [--m 8192 32768] [--out profiles/prefill_gemm.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd import ops
from distributed_llms_amd.ops import gemm

SHAPES = {"qkv_8b": (6144, 4096, False), "o_8b": (4096, 4096, False), "gate_up_8b": (28672, 4096, True),
          "down_8b": (4096, 14336, False)}


def timeit(fn, iters=10):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192, 32768])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for name, (n, k, sw) in SHAPES.items():
        w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            impls = {
                "blas": (lambda: ops.silu_mul(F.linear(x, w))) if sw else (lambda: F.linear(x, w)),
                "wide": lambda: gemm.linear_wide(x, w, splits=1, swiglu=sw, variant=4),
                "wide_grp": lambda: gemm.linear_wide(x, w, splits=1, swiglu=sw, variant=4 | 64),
            }
            for f in impls.values():
                f()
            torch.cuda.synchronize()
            res = {key: [] for key in impls}
            for _ in range(3):
                for key, f in impls.items():
                    res[key].append(timeit(f))
            t = {key: min(v) for key, v in res.items()}
            fl = 2.0 * m * n * k
            rows.append((name, m, t))
            print(f"{name:11s} {m:6d} " + " ".join(f"{key} {v*1e6:8.1f} us ({fl/v/1e15:4.2f} PF)" for key, v in t.items()),
                  flush=True)
            del x
        del w
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            f.write("| shape | M | hipBLASLt (+silu_mul) us | wide us | wide grouped us | grouped vs hipBLASLt |\n"
                    "|---|---|---|---|---|---|\n")
            for name, m, t in rows:
                f.write(f"| {name} | {m} | {t['blas']*1e6:.0f} | {t['wide']*1e6:.0f} | {t['wide_grp']*1e6:.0f} | "
                        f"{t['blas']/t['wide_grp']:.2f}x |\n")


if __name__ == "__main__":
    main()
