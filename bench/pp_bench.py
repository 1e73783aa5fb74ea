"""gemm_pp (ping-pong 256-row tiles) vs the engine's current GEMMs, Llama-3-8B projection shapes.

Decode (M = batch): every implementation runs as the engine runs it -- qkv materialised
(split-K + reduce), o / down deferred (slabs left for the fused norm), gate|up with the SwiGLU --
inside one HIP graph that rotates through > 768 MB of weight copies (each call streams its weight
from HBM, as a decode step does).  Prefill (M = tokens): hipBLASLt (F.linear, + silu_mul for
gate|up) vs gemm_pp with the grouped tile order and the fused SwiGLU, one weight copy (warm).
Interleaved rounds in one process, min over rounds (guide rule 24).

    python bench/pp_bench.py [--m 256] [--prefill 32768] [--shapes qkv o gate_up down]
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

SHAPES = {  # name: (N, K, swiglu, role)
    "qkv": (6144, 4096, False, "mat"), "o": (4096, 4096, False, "defer"),
    "gate_up": (28672, 4096, True, "swiglu"), "down": (4096, 14336, False, "defer"),
    "lm_head": (128256, 4096, False, "mat"),
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


def decode_impls(x, n, k, sw, role):
    defer = role == "defer"

    def wide(w):
        if sw:
            return gemm.linear_wide(x, w, swiglu=True)
        return gemm.linear_wide(x, w, defer=defer)

    impls = {"wide": wide}
    m = x.shape[0]
    for bn, vb in ((256, 0), (128, 1)):
        if n % bn:
            continue
        base = gemm.pp_splits(m, n, k, bn)
        for s in sorted({max(1, base // 2), base} | ({1, 2} if sw else set())):
            for nt in (0, 2, 64, 66):          # 64: schedule 2 (staging spread over the K-tile), 66: + nt
                v = vb | nt

                def f(w, s=s, v=v):
                    return gemm.linear_pp(x, w, splits=s, swiglu=sw, defer=defer, variant=v)
                impls[f"pp{bn}s{s}{ {0: '', 2: 'nt', 64: 'S2', 66: 'S2nt'}[nt] }"] = f
    return impls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--prefill", type=int, nargs="*", default=[32768])
    ap.add_argument("--shapes", nargs="+", default=["qkv", "o", "gate_up", "down"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--pf-variants", type=int, nargs="*", default=[], help="gemm_pf variants (8: nontemporal output stores)")
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in ([] if a.no_decode else a.shapes):
        n, k, sw, role = SHAPES[name]
        copies = max(2, -(-(768 << 20) // (n * k * 2)))
        ws = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            impls = decode_impls(x, n, k, sw, role)
            reps = max(copies, 8)
            graphs = {key: graph_of(f, ws, reps) for key, f in impls.items()}
            res = {key: [] for key in graphs}
            for _ in range(a.rounds):
                for key, g in graphs.items():
                    res[key].append(timeit(g.replay, a.iters) / reps)
            t = {key: min(v) * 1e6 for key, v in res.items()}
            best = min(t, key=t.get)
            print(f"decode {name:8s} M={m:4d} {role:6s} wide {t['wide']:7.1f} us | "
                  + " ".join(f"{key} {v:6.1f}" for key, v in t.items() if key != "wide")
                  + f" | best {best} {t[best]:.1f} ({t['wide'] / t[best]:.2f}x)", flush=True)
            del graphs
        del ws
        torch.cuda.empty_cache()
    for T in a.prefill or []:
        for name in a.shapes:
            n, k, sw, _ = SHAPES[name]
            if name == "lm_head":
                continue
            w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
            x = torch.randn(T, k, device="cuda").to(torch.bfloat16)
            impls = {"blas": (lambda w: ops.silu_mul(F.linear(x, w))) if sw else (lambda w: F.linear(x, w))}
            for bn, vb in ((256, 0), (128, 1)):
                if n % bn:
                    continue
                for grp in ((4, 68) if bn == 256 else (68,)):                    # grouped order; 68 = grouped + schedule 2
                    v = vb | grp
                    impls[f"pp{bn}g{'S2' if grp & 64 else ''}"] = (lambda w, v=v: gemm.linear_pp(
                        x, w, splits=1, swiglu=sw, variant=v))
            impls["pf"] = lambda w: gemm.linear_pf(x, w, swiglu=sw)   # persistent schedule 2
            for v in [u for u in a.pf_variants if u == 8]:
                impls[f"pf{v}"] = lambda w, v=v: gemm.linear_pf(x, w, swiglu=sw, variant=v)
            graphs = {key: graph_of(f, [w], 2) for key, f in impls.items()}
            res = {key: [] for key in graphs}
            for _ in range(a.rounds):
                for key, g in graphs.items():
                    res[key].append(timeit(g.replay, max(3, a.iters // 2)) / 2)
            t = {key: min(v) * 1e6 for key, v in res.items()}
            fl = 2.0 * T * n * k
            print(f"prefill {name:8s} T={T:6d} " + " ".join(f"{key} {fl / v / 1e6:5.0f}"
                                                           for key, v in t.items()) + " TF", flush=True)
            del graphs, x, w
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
