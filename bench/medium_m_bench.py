"""Medium-M GEMMs (257 <= M <= 2048: mixed prefill + decode steps, short prefills): which kernel?

Llama-3-8B projection shapes, every candidate the dispatcher could send them to:
  wide   gemm_wide (256 x 128 tiles, several row tiles, split-K over the CUs; partials reduced)
  pf     gemm_pf (persistent 256 x 256 tiles, dynamic tile queue)
  pp_sk  gemm_pp schedule 2 with split-K (256 x 256 tiles, K slices fill the CUs; reduced)
  blas   F.linear (hipBLASLt; + silu_mul for gate|up)
Weights rotate through copies totalling > 512 MB (each call streams its weight from HBM, as a
serving step does).  Median of interleaved rounds, us.  Advisor round 4: set the gemm_pf cutover
from measurements at these M, not from T = 8192 / 32768 tables.

    python bench/medium_m_bench.py [--m 320 512 768 1024 2048] [--shapes qkv o gate_up down]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd import knobs, ops
from distributed_llms_amd.ops import gemm

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False)}


def impls(n, k, sw):
    def wide(x, w):
        return gemm.linear_wide(x, w, swiglu=sw)

    def pf(x, w):
        return gemm.linear_pf(x, w, swiglu=sw)

    def pp_sk(x, w):
        m = x.shape[0]
        return gemm.linear_pp(x, w, splits=gemm.pp_splits(m, n, k), swiglu=sw, variant=gemm.PP_PREFILL_VARIANT)

    def blas(x, w):
        y = F.linear(x, w)
        return ops.silu_mul(y) if sw else y
    return {"wide": wide, "pf": pf, "pp_sk": pp_sk, "blas": blas}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[320, 384, 512, 640, 768, 1024, 1536, 2048])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    torch.manual_seed(0)
    print(f"{'shape':8s} {'M':>5s} " + " ".join(f"{k:>9s}" for k in ("wide", "pf", "pp_sk", "blas")) + "   best")
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, int((512 << 20) // (n * k * 2)) + 1)
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            fns = impls(n, k, sw)
            ok = {}
            for key, fn in fns.items():
                try:
                    fn(x, ws[0])
                    ok[key] = fn
                except Exception:          # noqa: BLE001 - a kernel that does not take the shape
                    pass
            res = {key: [] for key in ok}
            torch.cuda.synchronize()
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
            cells = " ".join(f"{med[key]:9.1f}" if key in med else f"{'-':>9s}" for key in ("wide", "pf", "pp_sk", "blas"))
            tf = 2.0 * m * n * k / (med[best] * 1e-6) / 1e12
            print(f"{name:8s} {m:5d} {cells}   {best} ({tf:.0f} TF/s)", flush=True)
        del ws


if __name__ == "__main__":
    main()
