"""FP8 W8A8 decode GEMM vs the bf16 engine GEMM, per Llama projection shape (ops/quant.py).

Cold weights (enough rotating copies that every call streams its weight from HBM, as each layer
does once per decode step), every implementation captured in one HIP graph of back-to-back
calls and replayed interleaved (launch overhead out, clocks shared).  Columns:
  bf16   the engine's bf16 path for the shape (wide kernel / hipBLASLt, ops.linear)
  fp8    quantize the activations (quant_fp8_rows) + gemm_wide_fp8, what the engine runs
  gemm   gemm_wide_fp8 alone on pre-quantized activations
    python bench/fp8_bench.py [--m 64 128 256] [--shapes qkv_8b ...] [--out profiles/fp8_gemm.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd import _ext, ops
from distributed_llms_amd.ops import gemm, quant

SHAPES = {  # name: (N, K, swiglu)
    "qkv_8b": (6144, 4096, False), "o_8b": (4096, 4096, False), "gate_up_8b": (28672, 4096, True),
    "down_8b": (4096, 14336, False),
    "qkv_70b": (10240, 8192, False), "o_70b": (8192, 8192, False), "gate_up_70b": (57344, 8192, True),
    "down_70b": (8192, 28672, False),
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


def gemm_only(xq, xs, w, m, n, k, sw, y, splits=0, bm=0, grp=False):
    s, bm0 = quant.fp8_plan(m, n, k, sw)
    if splits:
        s, bm0 = splits, bm
    bm = bm0
    ws = gemm._workspace(xq.device)
    v = (1 if m <= 256 else (4 | (64 if grp else 0))) | (bm << 8)
    _ext.kernels().gemm_wide_fp8(y.data_ptr(), xq.data_ptr(), xs.data_ptr(), w.q.data_ptr(), w.scale.data_ptr(),
                                 ws.data_ptr(), ws.numel(), m, n, k, s, 1 if sw else 0, v,
                                 torch.cuda.current_stream().cuda_stream)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[64, 128, 256])
    ap.add_argument("--shapes", nargs="+", default=["qkv_8b", "o_8b", "gate_up_8b", "down_8b"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--sweep", nargs="*", default=[], metavar="SPLITSxBM",
                    help="extra gemm-only configs, e.g. 4x0 8x0 8x128 (splits x row-tile override, 0 = default)")
    a = ap.parse_args()
    rows = []
    print(f"{'shape':12s} {'M':>5s} {'bf16_us':>8s} {'fp8_us':>8s} {'gemm_us':>8s} {'speedup':>8s} {'fp8_TF':>7s}",
          flush=True)
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, -(-(768 << 20) // (n * k)))            # > the 256 MiB MALL, fp8 bytes
        wb = [(torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(min(copies, 8))]
        w8 = [quant.quantize_weight(w) for w in wb]
        while len(w8) < copies:                                 # extra fp8 copies (bf16 rotates over fewer)
            w8.append(quant.Fp8Weight(w8[len(w8) % len(wb)].q.clone(), w8[len(w8) % len(wb)].scale.clone()))
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            xq, xs = quant.quantize_rows(x)
            y = torch.empty(m, n // 2 if sw else n, dtype=torch.bfloat16, device="cuda")
            impls = {
                "bf16": (lambda i: ops.linear_swiglu(x, wb[i % len(wb)])) if sw else
                        (lambda i: ops.linear(x, wb[i % len(wb)])),
                "fp8": lambda i: quant.linear_fp8(x, w8[i % len(w8)], swiglu=sw),
                "gemm": lambda i: gemm_only(xq, xs, w8[i % len(w8)], m, n, k, sw, y),
                "quant": lambda i: quant.quantize_rows(x),
                **({"grp": lambda i: gemm_only(xq, xs, w8[i % len(w8)], m, n, k, sw, y, grp=True)} if m > 256 else {}),
                **{f"s{c}": (lambda i, c=c: gemm_only(xq, xs, w8[i % len(w8)], m, n, k, sw, y,
                                                      *map(int, c.split("x")))) for c in a.sweep
                   if int(c.split("x")[0]) * m * n <= gemm._workspace(x.device).numel()},
            }
            reps = max(len(w8), 8)
            graphs = {}
            for key, f in impls.items():
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    for i in range(reps):
                        f(i)
                torch.cuda.current_stream().wait_stream(st)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for i in range(reps):
                        f(i)
                graphs[key] = g
            for g in graphs.values():
                g.replay()
            res = {key: [] for key in graphs}
            for _ in range(3):
                for key, g in graphs.items():
                    res[key].append(timeit(g.replay, max(3, a.iters // 5)) / reps)
            t = {key: min(v) for key, v in res.items()}
            tf = 2.0 * m * n * k / t["gemm"] / 1e12
            rows.append((name, m, t["bf16"], t["fp8"], t["gemm"]))
            print(f"{name:12s} {m:5d} {t['bf16']*1e6:8.1f} {t['fp8']*1e6:8.1f} {t['gemm']*1e6:8.1f} "
                  f"{t['bf16']/t['fp8']:8.2f} {tf:7.0f}  quant {t['quant']*1e6:5.1f} "
                  + (f"grouped {t['grp']*1e6:7.1f} " if "grp" in t else "")
                  + " ".join(f"{c} {t['s' + c]*1e6:6.1f}" for c in a.sweep if "s" + c in t), flush=True)
        del wb, w8
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            f.write("| shape | M | bf16 engine us | fp8 (quant + GEMM) us | fp8 GEMM us | speedup | fp8 GEMM TFLOP/s |\n"
                    "|---|---|---|---|---|---|---|\n")
            for name, m, tb, t8, tg in rows:
                n, k, _ = SHAPES[name]
                f.write(f"| {name} | {m} | {tb*1e6:.1f} | {t8*1e6:.1f} | {tg*1e6:.1f} | {tb/t8:.2f}x | "
                        f"{2.0*m*n*k/tg/1e12:.0f} |\n")


if __name__ == "__main__":
    main()
