"""Medium-M sweep of gemm_wide's row tile and K split (review item: medium-M GEMM path).

For each Llama-3-8B projection at M in --m: gemm_wide at row tiles 128 / 192 / 256 and K splits
1-4 (split results reduced, as linear_wide does without ``defer``), against what ops.gemm.linear
dispatches today.  Weights rotate through > 512 MB of copies (each call streams its weight from
HBM).  Median of interleaved rounds, us.

    python bench/debug/medium_m_sweep.py [--m 384 512 768 1024] [--shapes qkv o gate_up down]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd import knobs, ops
from distributed_llms_amd.ops import gemm

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False), "head": (128256, 4096, False),
          "qkv70": (10240, 8192, False), "o70": (8192, 8192, False), "gate_up70": (57344, 8192, True),
          "down70": (8192, 28672, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[384, 512, 768, 1024])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--bms", type=int, nargs="+", default=[128, 256])
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--pp", nargs="*", default=[],
                    help="gemm_pp candidates BN:SPLITS[:nt], e.g. 128:1:nt 256:2 (schedule 2)")
    ap.add_argument("--no-wide", action="store_true", help="skip the gemm_wide grid")
    ap.add_argument("--sq", type=int, nargs="*", default=[], help="gemm_sq (256 x 256 tiles) at these K splits")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, int((512 << 20) // (n * k * 2)) + 1)
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            fns = {}
            if sw:
                fns["dispatch"] = lambda x, w: ops.linear_swiglu(x, w)
            else:
                fns["dispatch"] = lambda x, w: gemm.linear(x, w)
            for spec in a.pp:
                f = spec.split(":")
                bn, sp, nt = int(f[0]), int(f[1]), len(f) > 2 and f[2] == "nt"
                var = 64 | (1 if bn == 128 else 0) | (2 if nt else 0)
                fns[f"pp{bn}s{sp}{'nt' if nt else ''}"] = (lambda sp, var: lambda x, w: gemm.linear_pp(
                    x, w, splits=sp, swiglu=sw, variant=var))(sp, var)
            for sp in a.sq:
                fns[f"sq{sp}"] = (lambda sp: lambda x, w: gemm.linear_sq(x, w, splits=sp, swiglu=sw))(sp)
            for bm in ([] if a.no_wide else a.bms):
                for s in a.splits:
                    v = knobs.K.wide_variant_split if s > 1 else knobs.K.wide_variant
                    fns[f"w{bm}s{s}"] = (lambda bm, s, v: lambda x, w: gemm.linear_wide(
                        x, w, splits=s, swiglu=sw, variant=v | (bm << 8)))(bm, s, v)
            ok = {}
            ref = None
            for key, fn in fns.items():
                try:
                    y = fn(x, ws[0])
                    torch.cuda.synchronize()
                except Exception as e:      # noqa: BLE001 - a configuration the kernel does not take
                    print(f"  {name} M={m} {key}: {type(e).__name__}: {e}", flush=True)
                    continue
                if ref is None:
                    ref = y.float()
                else:
                    err = (y.float() - ref).abs().max().item()
                    if err > 0.05 * ref.abs().max().item() + 1e-3:
                        print(f"  {name} M={m} {key}: max diff {err:.3g} -- skipped", flush=True)
                        continue
                ok[key] = fn
            res = {key: [] for key in ok}
            for _ in range(a.rounds):
                for key, fn in ok.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(a.calls):
                        fn(x, ws[i % copies])
                    e1.record()
                    e1.synchronize()
                    res[key].append(e0.elapsed_time(e1) * 1e3 / a.calls)
            med = {key: statistics.median(v) for key, v in res.items()}
            best = min(med, key=med.get)
            tf = 2.0 * m * n * k / (med[best] * 1e-6) / 1e12
            cells = "  ".join(f"{key} {t:.1f}" for key, t in med.items())
            print(f"{name:8s} M={m:5d}  {cells}   best {best} ({tf:.0f} TF/s)", flush=True)
        del ws


if __name__ == "__main__":
    main()
