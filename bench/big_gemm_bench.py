"""gemm_big (256 x 256 x 32 tile, one 128 x 128 wave per SIMD) vs the engine's wide / sq kernel.

Graph-captured back-to-back calls over rotating weight copies (> 768 MB: every call streams its
weights from HBM), us per call, Llama-3-8B decode shapes:

    python bench/big_gemm_bench.py [--m 256] [--splits 1 2 4 8]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import gemm

SHAPES = {"gate_up_8b": (28672, 4096, True), "down_8b": (4096, 14336, False), "qkv_8b": (6144, 4096, False),
          "o_8b": (4096, 4096, False), "lm_head_8b": (128256, 4096, False)}


def timeit(g, iters=5):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    a = ap.parse_args()
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, -(-(768 << 20) // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            impls = {"engine": lambda w: gemm.linear_wide(x, w, swiglu=sw)}
            for s in a.splits:
                if sw and s == 1:
                    continue
                if (k // 32) < s or (s > 1 and s * m * n > gemm._workspace(x.device).numel()):
                    continue
                impls[f"big_s{s}"] = (lambda w, s=s: gemm.linear_big(x, w, splits=s, swiglu=sw))
            reps = max(copies, 8)
            res = {}
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
                g.replay()
                res[key] = min(timeit(g) for _ in range(3)) / reps
            print(f"{name:11s} M={m:4d} " + "  ".join(f"{k_} {v * 1e6:6.1f}" for k_, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
