"""Stream-K gemm_wide vs the unsplit kernel on the decode gate|up (and a plain projection).

Weights rotate through > 512 MB of copies (cold, as in serving).  Median us of interleaved rounds.

    python bench/debug/streamk_bench.py [--m 64 128 256]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd.ops import gemm

SHAPES = {"gate_up_8b": (28672, 4096, True), "gate_up_70b": (57344, 8192, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[64, 128, 256])
    ap.add_argument("--shapes", nargs="+", default=["gate_up_8b"])
    ap.add_argument("--grids", type=int, nargs="+", default=[256, 240, 224])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in a.shapes:
        n, k, sw = SHAPES[name]
        copies = max(2, int((512 << 20) // (n * k * 2)) + 1)
        ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
            fns = {"wide": lambda w: gemm.linear_wide(x, w, splits=1, swiglu=sw)}
            for g in a.grids:
                fns[f"sk{g}"] = lambda w, g=g: gemm.linear_wide_sk(x, w, swiglu=sw, grid=g)
            fns["sk256_nopart"] = lambda w: gemm.linear_wide_sk(x, w, swiglu=sw, grid=256, test=2)
            res = {key: [] for key in fns}
            for fn in fns.values():
                fn(ws[0])
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for key, fn in fns.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for i in range(a.calls):
                        fn(ws[i % copies])
                    e1.record()
                    e1.synchronize()
                    res[key].append(e0.elapsed_time(e1) * 1e3 / a.calls)
            sk = gemm._sk_block(x.device).cpu()
            print(f"{name} M={m:4d}  " + "  ".join(f"{key} {statistics.median(v):6.1f}" for key, v in res.items())
                  + f"   steals {int(sk[3])}", flush=True)
            assert int(gemm._sk_block(x.device)[2]) == 0
        del ws


if __name__ == "__main__":
    main()
