"""Decode GEMMs (M = 256, engine dispatch) with their weights cold (rotating > 768 MB of copies:
every call streams from HBM) vs warm (one copy, re-read back to back: resident in the 256 MB
Infinity Cache when it fits).  Measures what a weight prefetch into the Infinity Cache could buy.

    python bench/mall_bench.py [--shapes qkv o gate_up down]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import gemm

SHAPES = {"qkv": (6144, 4096, False, False), "o": (4096, 4096, False, True),
          "gate_up": (28672, 4096, True, False), "down": (4096, 14336, False, True), "head": (128256, 4096, False, False)}


def run(x, w, sw, defer):
    if sw:
        return gemm.linear_swiglu(x, w)
    return gemm.linear(x, w, defer=defer)


def graph_of(fn, ws, reps):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for i in range(reps):
            fn(ws[i % len(ws)])
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for i in range(reps):
            fn(ws[i % len(ws)])
    return g


def timeit(g, iters, reps):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["qkv", "o", "gate_up", "down", "head"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--knobs", default="", help="kernel knobs for this run (knobs.parse syntax)")
    a = ap.parse_args()
    from distributed_llms_amd import knobs
    knobs.update(knobs.parse(a.knobs))
    torch.manual_seed(0)
    x = torch.randn(256, 4096, device="cuda").to(torch.bfloat16)
    for name in a.shapes:
        n, k, sw, defer = SHAPES[name]
        xx = torch.randn(256, k, device="cuda").to(torch.bfloat16) if k != 4096 else x
        copies = max(2, -(-(768 << 20) // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        reps = max(copies, 8)
        gc = graph_of(lambda w: run(xx, w, sw, defer), ws, reps)
        gw = graph_of(lambda w: run(xx, w, sw, defer), ws[:1], reps)
        cold, warm = [], []
        for _ in range(a.rounds):
            cold.append(timeit(gc, 5, reps))
            warm.append(timeit(gw, 5, reps))
        c, w_ = min(cold), min(warm)
        mb = n * k * 2 / 1e6
        print(f"{name:8s} {mb:7.1f} MB  cold {c:7.1f} us ({mb / c:.2f} TB/s)  warm {w_:7.1f} us ({mb / w_:.2f} TB/s)"
              f"  warm/cold {w_ / c:.2f}", flush=True)
        del gc, gw, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
