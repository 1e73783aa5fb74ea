"""Decode GEMM microbenchmark: the engine's hand-written wide-M MFMA kernel (gemm_wide.hip, plus
gemm_sq.hip with --sq and extra variants) vs hipBLASLt (torch), cold (rotating > 768 MB of weight
copies, in-engine-like) or --warm, each implementation graph-captured, interleaved in one process
(CDNA guide rule 24).  Reports time, weight-streaming TB/s and TFLOP/s.
    python bench/gemm_bench.py [--m 64 256] [--shapes qkv_8b gate_up_8b]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd import knobs, ops
from distributed_llms_amd.ops import gemm

SHAPES = {  # name: (N, K, swiglu)
    "qkv_8b": (6144, 4096, False), "o_8b": (4096, 4096, False), "gate_up_8b": (28672, 4096, True),
    "down_8b": (4096, 14336, False), "lm_head_8b": (128256, 4096, False),
    "qkv_70b": (10240, 8192, False), "down_70b": (8192, 28672, False),
    "o_70b": (8192, 8192, False), "gate_up_70b": (57344, 8192, True),
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
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16, 64, 256])
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--warm", action="store_true", help="no cache flush between calls (in-engine-like)")
    ap.add_argument("--splits", type=int, default=0)
    ap.add_argument("--variants", type=int, nargs="*", default=[0],
                    help="extra gemm_wide variants timed beside the engine's choice")
    ap.add_argument("--sq", action="store_true", help="also time the 256 x 256-tile gemm_sq kernel")
    ap.add_argument("--sq-alt", type=int, default=0, help="--sq: second gemm_sq variant timed (sq0)")
    a = ap.parse_args()
    return wide(a)


def wide(a):
    """Comparison.  Cold = rotate through enough weight copies (> 768 MB) that every call
    streams its weight from HBM, with no dirty flush buffer competing for write-back (in-engine-like:
    each layer's weights are read once per step).  --warm = one copy (MALL-resident)."""
    print(f"{'shape':12s} {'M':>4s} {'wide_us':>8s} {'TB/s':>6s} {'TF':>6s} {'blas_us':>8s} "
          f"{'vs_blas':>8s}  ({'warm' if a.warm else 'cold, rotating weights'})")
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = 1 if a.warm else max(2, -(-(768 << 20) // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            # one HIP graph per implementation: `copies` back-to-back calls, each on its own weight
            # copy (launch overhead out of the measurement, like the engine's captured decode step)
            split = (a.splits or gemm.wide_splits(m, n, k, sw)) > 1
            wv = knobs.K.wide_variant_split if split else knobs.K.wide_variant     # the engine's choice
            impls = {
                "wide": lambda w: gemm.linear_wide(x, w, splits=a.splits, swiglu=sw, variant=wv),
                **{f"v{v}": (lambda w, v=v: gemm.linear_wide(x, w, splits=a.splits, swiglu=sw, variant=v))
                   for v in a.variants},
                **({"sq": lambda w: gemm.linear_sq(x, w, swiglu=sw, variant=4),
                    "sq0": lambda w: gemm.linear_sq(x, w, swiglu=sw, variant=a.sq_alt)} if a.sq and n % 256 == 0 else {}),
                "blas": (lambda w: ops.silu_mul(F.linear(x, w))) if sw else (lambda w: F.linear(x, w)),
            }
            reps = max(copies, 8)
            graphs = {}
            for key, f in impls.items():
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    for i in range(reps):
                        f(ws[i % copies])
                torch.cuda.current_stream().wait_stream(st)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for i in range(reps):
                        f(ws[i % copies])
                graphs[key] = g
            for g in graphs.values():
                g.replay()
            res = {key: [] for key in graphs}
            for _ in range(3):
                for key, g in graphs.items():
                    res[key].append(timeit(g.replay, max(3, a.iters // 5)) / reps)
            t = {key: min(v) for key, v in res.items()}
            byt, fl_ = n * k * 2, 2.0 * m * n * k
            print(f"{name:12s} {m:4d} {t['wide']*1e6:8.1f} {byt/t['wide']/1e12:6.2f} {fl_/t['wide']/1e12:6.0f} "
                  f"{t['blas']*1e6:8.1f} {t['blas']/t['wide']:8.2f} "
                  + " ".join(f"v{v} {t[f'v{v}']*1e6:6.1f}" for v in a.variants)
                  + (f" sq {t['sq']*1e6:6.1f} ({t['wide']/t['sq']:.2f}x) sq0 {t['sq0']*1e6:6.1f}" if "sq" in t else ""),
                  flush=True)


if __name__ == "__main__":
    main()
