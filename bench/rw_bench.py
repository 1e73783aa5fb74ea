"""gemm_rw (register-weight decode GEMM) vs gemm_wide, Llama-3-8B / 70B decode projection shapes.

Each implementation runs as the engine runs it (qkv materialised, o / down deferred split-K slabs,
gate|up with the SwiGLU) inside one HIP graph that rotates through > 768 MB of weight copies, so
every call streams its weight from HBM as a decode step does.  Interleaved rounds, min over rounds.

    python bench/rw_bench.py [--m 256] [--shapes qkv o gate_up down] [--ns 3 4 5] [--packed 0 1]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import gemm

SHAPES = {  # name: (N, K, swiglu, role)
    "qkv": (6144, 4096, False, "mat"), "o": (4096, 4096, False, "defer"),
    "gate_up": (28672, 4096, True, "swiglu"), "down": (4096, 14336, False, "defer"),
    "qkv70": (10240, 8192, False, "mat"), "o70": (8192, 8192, False, "defer"),
    "gate_up70": (57344, 8192, True, "swiglu"), "down70": (8192, 28672, False, "defer"),
    "head": (128256, 4096, False, "mat"),
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--shapes", nargs="+", default=["qkv", "o", "gate_up", "down", "head"])
    ap.add_argument("--ns", type=int, nargs="+", default=[0], help="ring depths (0: the row tile's default)")
    ap.add_argument("--splits", type=int, nargs="*", default=[])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--packed", type=int, nargs="+", default=[0, 1], help="0: nn.Linear layout, 1: pack_rw")
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in a.shapes:
        n, k, sw, role = SHAPES[name]
        defer = role == "defer"
        copies = max(2, -(-(768 << 20) // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wps = [gemm.pack_rw(w, sw) for w in ws] if 1 in a.packed else []
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            impls = {}
            if name == "head":       # the engine's LM head today: gemm_pp schedule 2, nt weights
                impls["wide"] = (lambda w: gemm.linear_pp(x, w, splits=1, variant=gemm.PP_HEAD_VARIANT), ws)
            elif m <= 512:
                impls["wide"] = ((lambda w: gemm.linear_wide(x, w, swiglu=True)) if sw else
                                 (lambda w: gemm.linear_wide(x, w, defer=defer)), ws)
            base = gemm.rw_splits(m, n, k, sw)
            for s in sorted({base} | set(a.splits)):
                for ns in a.ns:
                    for pk in a.packed:
                        impls[f"rw{ns}s{s}{'p' if pk else ''}"] = (
                            lambda w, s=s, ns=ns, pk=pk: gemm.linear_rw(x, w, splits=s, swiglu=sw, defer=defer,
                                                                        variant=ns, packed=bool(pk)),
                            wps if pk else ws)
            reps = max(copies, 8)
            graphs = {key: graph_of(f, wl, reps) for key, (f, wl) in impls.items()}
            res = {key: [] for key in graphs}
            for _ in range(a.rounds):
                for key, g in graphs.items():
                    res[key].append(timeit(g.replay, a.iters) / reps)
            t = {key: min(v) * 1e6 for key, v in res.items()}
            best = min(t, key=t.get)
            wb = n * k * 2
            print(f"decode {name:9s} M={m:4d} " + " ".join(f"{key} {v:6.1f}" for key, v in t.items())
                  + f" | best {best} {t[best]:.1f} us = {wb / t[best] / 1e6:.2f} TB/s"
                  + (f" ({t['wide'] / t[best]:.2f}x wide)" if "wide" in t else ""), flush=True)
            del graphs
        del ws, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
