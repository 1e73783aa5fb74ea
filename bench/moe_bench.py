"""Mixtral MoE layer microbenchmark (decode-sized token counts) on one MI355X.

Times the HIP path (route + grouped gate|up/SwiGLU + grouped down + combine) against a
per-expert hipBLASLt loop (gather, F.linear per expert, host-side counts), and reports the
expert-weight streaming rate (bytes of the experts that received tokens / time).

    python bench/moe_bench.py [--tokens 16 64 128 256] [--iters 20]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd import _ext, knobs, ops
from distributed_llms_amd.ops import moe


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


def blas_loop(x, wr, wgu, wd, top_k):
    logits = F.linear(x, wr).float()
    p = torch.softmax(logits, -1)
    tw, tid = p.topk(top_k, -1)
    tw = tw / tw.sum(-1, keepdim=True)
    out = torch.zeros_like(x, dtype=torch.float32)
    for e in range(wgu.shape[0]):
        rows, j = (tid == e).nonzero(as_tuple=True)
        if rows.numel() == 0:
            continue
        h = F.linear(x[rows], wgu[e])
        i = h.shape[-1] // 2
        y = F.linear(F.silu(h[:, :i]) * h[:, i:], wd[e])
        out.index_add_(0, rows, y.float() * tw[rows, j, None])
    return out.to(x.dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="+", default=[16, 64, 128, 256])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--top-k", type=int, default=2)
    ap.add_argument("--variants", type=int, nargs="*", default=[1, 2, 3, 4, 5, 6],
                    help="also time each forced grouped-kernel variant (csrc/kernels/moe.hip)")
    a = ap.parse_args()
    _ext.kernels()
    torch.manual_seed(0)
    h, i, e = a.hidden, a.inter, a.experts
    dev = "cuda"
    wr = (torch.randn(e, h, device=dev) * 0.02).to(torch.bfloat16)
    wgu = (torch.randn(e, 2 * i, h, device=dev) * 0.02).to(torch.bfloat16)
    wd = (torch.randn(e, h, i, device=dev) * 0.02).to(torch.bfloat16)
    print(f"{'T':>5s} {'active':>6s} {'hip_us':>9s} {'hip_TB/s':>9s} {'blas_us':>9s} {'blas_TB/s':>9s} {'speedup':>8s} {'max_err':>8s}")
    for t in a.tokens:
        x = torch.randn(t, h, device=dev).to(torch.bfloat16)
        tid = torch.softmax(F.linear(x, wr).float(), -1).topk(a.top_k, -1).indices
        active = int(torch.unique(tid).numel())
        nbytes = active * 3 * h * i * 2
        f_hip = lambda: moe.forward(x, wr, wgu, wd, a.top_k)   # noqa: E731
        f_blas = lambda: blas_loop(x, wr, wgu, wd, a.top_k)    # noqa: E731
        f_hip(), f_blas()
        t_hip = [timeit(f_hip, a.iters)]
        t_blas = [timeit(f_blas, a.iters)]
        t_hip.append(timeit(f_hip, a.iters))
        th, tb = min(t_hip), t_blas[0]
        err = (f_hip().float() - f_blas().float()).abs().max().item()
        print(f"{t:5d} {active:6d} {th * 1e6:9.1f} {nbytes / th / 1e12:9.2f} {tb * 1e6:9.1f} {nbytes / tb / 1e12:9.2f} "
              f"{tb / th:8.2f} {err:8.4f}", flush=True)
        if t <= moe.GROUPED_MAX_TOKENS:
            knobs.K.moe_deep_ring = False
            f_hip()
            ts = timeit(f_hip, a.iters)
            knobs.K.moe_deep_ring = True
            print(f"      3-slot ring: {ts * 1e6:.1f} us ({nbytes / ts / 1e12:.2f} TB/s)", flush=True)
        if t <= moe.GROUPED_MAX_TOKENS and a.variants:
            row = []
            for v in a.variants:
                knobs.K.moe_variant = v
                f_hip()
                tv = timeit(f_hip, a.iters)
                e2 = (f_hip().float() - f_blas().float()).abs().max().item()
                row.append(f"v{v}={tv * 1e6:.0f}us({nbytes / tv / 1e12:.2f}TB/s{'' if e2 < 0.1 else ' BAD'})")
            knobs.K.moe_variant = 0
            print("      variants: " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
