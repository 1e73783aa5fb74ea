"""M = 256 decode projections: gemm_wide (256 x 128 tiles, split-K) vs gemm_pp schedule 2
(256 x 256 tiles, split-K), kernel alone (partials left in the workspace) and with the reduce.

Llama-3-8B shapes; weights rotate through > 512 MB of copies so every call streams its weight
from HBM as a serving step does.  Median of interleaved rounds, us.

    python bench/debug/decode_pp_split.py [--m 256] [--splits 2 4 8]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd import _ext
from distributed_llms_amd.ops import gemm

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4, 8, 16])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--extra", type=int, nargs="*", default=[],
                    help="extra gemm_pp variant bits to try (added to schedule 2)")
    a = ap.parse_args()
    torch.manual_seed(0)
    K_ = _ext.kernels()
    stream = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, int((512 << 20) // (n * k * 2)) + 1)
        ws_ = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            wsp = gemm._workspace(x.device)
            y = torch.empty(m, n // 2 if sw else n, dtype=torch.bfloat16, device="cuda")
            fns = {}
            fns["wide"] = lambda w: gemm.linear_wide(x, w, swiglu=sw, defer=not sw)
            ks = k // 64
            for s in a.splits:
                if s > 1 and (ks // s < 2 or (n // 256) * s > 512):
                    continue
                for extra in [0] + a.extra:
                    var = 64 | extra
                    tag = f"pp{s}" + (f"v{extra}" if extra else "")
                    if s == 1:
                        fns[tag] = (lambda w, var=var: K_.gemm_pp(y.data_ptr(), x.data_ptr(), w.data_ptr(), wsp.data_ptr(),
                                                                  wsp.numel(), m, n, k, 1, 1 if sw else 0, var, stream()))
                    else:
                        fns[tag + "k"] = (lambda w, s=s, var=var: K_.gemm_pp(0, x.data_ptr(), w.data_ptr(), wsp.data_ptr(), wsp.numel(),
                                                                            m, n, k, s, 2, var, stream()))
                        if sw:
                            fns[tag + "r"] = (lambda w, s=s, var=var: gemm.linear_pp(x, w, splits=s, swiglu=True, variant=var))
            res = {key: [] for key in fns}
            for fn in fns.values():
                fn(ws_[0])
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for key, fn in fns.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(a.calls):
                        fn(ws_[i % copies])
                    e1.record()
                    e1.synchronize()
                    res[key].append(e0.elapsed_time(e1) * 1e3 / a.calls)
            cells = "  ".join(f"{key} {statistics.median(v):.1f}" for key, v in res.items())
            print(f"{name:8s} M={m:4d}  {cells}", flush=True)
        del ws_


if __name__ == "__main__":
    main()
