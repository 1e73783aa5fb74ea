"""Decode GEMMs with weights cold (streamed from HBM) vs warm (resident in the 256 MB Infinity
Cache): the ceiling of any scheme that pulls the next GEMM's weights into the cache early.

    python bench/debug/warm_vs_cold_gemm.py

Llama-3-8B projections at M = 256 through the engine's dispatch (gemm_wide / gemm_sq):
cold = weights rotate through copies totalling > 1 GB (each call's weight was evicted by the
others); warm = the same weight every call (after the first, it is served from the cache).
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd import ops


def _time(fn, n=30):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3


def main():
    torch.manual_seed(0)
    m = 256
    shapes = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
              "down": (4096, 14336, False), "lm_head": (128256, 4096, False)}
    for name, (n, k, sw) in shapes.items():
        x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        copies = max(2, int((1 << 30) // (n * k * 2)) + 1)
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        it = [0]

        def call(w):
            return ops.linear_swiglu(x, w) if sw else ops.linear(x, w)

        def cold():
            it[0] += 1
            call(ws[it[0] % copies])

        call(ws[0])
        torch.cuda.synchronize()
        tc = _time(cold)
        tw = _time(lambda: call(ws[0]))
        mb = n * k * 2 / 1e6
        print(f"{name:8s} {mb:7.1f} MB  cold {tc:7.1f} us ({mb / tc:5.2f} TB/s)  warm {tw:7.1f} us "
              f"({mb / tw:5.2f} TB/s)  warm/cold {tw / tc:.2f}", flush=True)
        del ws


if __name__ == "__main__":
    main()
