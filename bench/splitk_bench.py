"""Split-K slab consumers (csrc/kernels/splitk.hip) at the decode shapes of Llama-3-8B / 70B:
splitk_add_rms_norm (o / down epilogue) and splitk_reduce (qkv), graph-captured, us per call.
Each call reads its own slab copy (rotating buffers > 256 MB, so slabs come from HBM like an
engine step whose slabs were written a GEMM earlier... or from MALL with --warm).

    python bench/splitk_bench.py [--warm]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd import _ext

CASES = [  # name, kind, M, N, S
    ("o/down 8B", "norm", 256, 4096, 8), ("o/down 8B M64", "norm", 64, 4096, 8),
    ("o/down 70B", "norm", 256, 8192, 8), ("qkv 8B", "reduce", 256, 6144, 5),
    ("qkv 70B", "reduce", 256, 10240, 4),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", action="store_true")
    ap.add_argument("--reps", type=int, default=32)
    a = ap.parse_args()
    k = _ext.kernels()
    dev = torch.device("cuda")
    for name, kind, m, n, s in CASES:
        slab_b = s * m * n * 2                         # f16 slabs
        copies = 1 if a.warm else max(2, (256 << 20) // slab_b + 1)
        ws = [torch.randn(s * m * n, device=dev).to(torch.float16) for _ in range(copies)]
        res = torch.randn(m, n, device=dev).to(torch.bfloat16)
        w = torch.randn(n, device=dev).to(torch.bfloat16)
        y = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

        def call(i):
            st = torch.cuda.current_stream().cuda_stream
            if kind == "norm":
                k.splitk_add_rms_norm(y.data_ptr(), res.data_ptr(), ws[i % copies].data_ptr(), s, m, n, w.data_ptr(),
                                      1e-5, st)
            else:
                k.splitk_reduce(y.data_ptr(), ws[i % copies].data_ptr(), 0, s, m, n, st)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for i in range(a.reps):
                call(i)
        torch.cuda.current_stream().wait_stream(st)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for i in range(a.reps):
                call(i)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.reps)
        t = statistics.median(ts)
        byt = slab_b + (3 if kind == "norm" else 1) * m * n * 2
        print(f"{name:14s} {kind:6s} M={m:4d} N={n:6d} S={s}: {t:6.2f} us  {byt / t / 1e6:5.2f} TB/s", flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
