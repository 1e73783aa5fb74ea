"""Does hipBLASLt pick a different (slower) kernel for F.linear under HIP-graph capture?

Times the decode GEMM shapes eager vs graph-replayed, and the LM head split in N-chunks.
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F


def t_eager(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def t_graph(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    return t_eager(g.replay, iters)


def main():
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    print(f"{'shape':8s} {'M':>4s} {'eager_us':>9s} {'graph_us':>9s} {'TB/s(e)':>8s} {'TB/s(g)':>8s}")
    for name, (n, k) in shapes.items():
        w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
        for m in (64, 128, 256):
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            fn = lambda: F.linear(x, w)
            te, tg = t_eager(fn), t_graph(fn)
            print(f"{name:8s} {m:4d} {te:9.1f} {tg:9.1f} {n*k*2/te/1e6:8.2f} {n*k*2/tg/1e6:8.2f}", flush=True)
    w = (torch.randn(128256, 4096, device="cuda") * 0.02).to(torch.bfloat16)
    for m in (64, 128, 256):
        x = torch.randn(m, 4096, device="cuda").to(torch.bfloat16)
        for chunks in (2, 4, 8):
            ws = list(torch.chunk(w, chunks, 0))
            out = torch.empty(m, 128256, device="cuda", dtype=torch.bfloat16)
            def fn():
                o = 0
                for wc in ws:
                    torch.matmul(x, wc.t(), out=out[:, o:o + wc.shape[0]]) if False else out[:, o:o + wc.shape[0]].copy_(F.linear(x, wc))
                    o += wc.shape[0]
            te, tg = t_eager(fn), t_graph(fn)
            print(f"lmhead/{chunks} {m:4d} {te:9.1f} {tg:9.1f}", flush=True)


if __name__ == "__main__":
    main()
