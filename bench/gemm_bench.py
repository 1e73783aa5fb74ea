"""Decode GEMM microbenchmark: hand-written skinny MFMA kernel vs hipBLASLt (torch).

Reports per-shape time and effective weight-streaming bandwidth (weight bytes / time),
interleaving the two implementations in one process (CDNA guide rule 24).
    python bench/gemm_bench.py [--m 64] [--iters 50]
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

SHAPES = {  # name: (N, K, swiglu)
    "qkv_8b": (6144, 4096, False), "o_8b": (4096, 4096, False), "gate_up_8b": (28672, 4096, True),
    "down_8b": (4096, 14336, False), "lm_head_8b": (128256, 4096, False),
    "qkv_70b": (10240, 8192, False), "down_70b": (8192, 28672, False),
}


def timeit(fn, iters):
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
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16, 64])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--tiled", action="store_true", help="compare the split-K tiled kernel instead")
    a = ap.parse_args()
    # a scratch buffer larger than the 256 MiB Infinity Cache to flush it between calls
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    print(f"{'shape':12s} {'M':>4s} {'ours_us':>9s} {'ours_TB/s':>10s} {'blas_us':>9s} {'blas_TB/s':>10s} {'speedup':>8s}")
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            if a.tiled:
                ours = lambda: (flush.zero_(), gemm.linear_tiled(x, w, swiglu=sw))
                blas = (lambda: (flush.zero_(), ops.silu_mul(F.linear(x, w)))) if sw else (lambda: (flush.zero_(), F.linear(x, w)))
            elif sw:
                ours = lambda: (flush.zero_(), gemm.linear_swiglu(x, w, force_skinny=True))
                blas = lambda: (flush.zero_(), ops.silu_mul(F.linear(x, w)))
            else:
                ours = lambda: (flush.zero_(), gemm.linear(x, w, force_skinny=True))
                blas = lambda: (flush.zero_(), F.linear(x, w))
            base = timeit(lambda: flush.zero_(), a.iters)
            for _ in range(3):
                ours(); blas()
            to, tb = [], []
            for _ in range(3):
                to.append(timeit(ours, a.iters) - base)
                tb.append(timeit(blas, a.iters) - base)
            to, tb = min(to), min(tb)
            byt = n * k * 2
            print(f"{name:12s} {m:4d} {to*1e6:9.1f} {byt/to/1e12:10.2f} {tb*1e6:9.1f} {byt/tb/1e12:10.2f} {tb/to:8.2f}",
                  flush=True)


if __name__ == "__main__":
    main()
