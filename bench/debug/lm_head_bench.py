"""Decode LM head (Llama-3-8B: 128,256 x 4,096, M = 256) on each candidate kernel, us per call over
rotating weight copies (each call streams its weight from HBM, as a decode step does).

    python bench/debug/lm_head_bench.py
"""
import os
import statistics
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "scripts"))     # hwq_probe.SpinnerProc (also in spawned children)

import torch

from distributed_llms_amd.ops import gemm


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--spinner", action="store_true",
                    help="time beside a 4-workgroup receive (20 KiB LDS each) spinning in another process")
    a = ap.parse_args()
    torch.manual_seed(0)
    m, n, k = 256, 128256, 4096
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(3)]
    it = [0]
    cands = {
        "pp_head (shipped)": lambda w: gemm.linear_pp(x, w, splits=1, variant=gemm.PP_HEAD_VARIANT),
        "pp_sched2_default_policy": lambda w: gemm.linear_pp(x, w, splits=1, variant=64),
        "pf_static": lambda w: gemm.linear_pf(x, w),
        "pf_dynamic": lambda w: gemm.linear_pf(x, w, variant=16),
        "wide/sq": lambda w: gemm.linear_wide(x, w),
        "pp_head_128col": lambda w: gemm.linear_pp(x, w, splits=1, variant=gemm.PP_HEAD_VARIANT | 1),
    }
    res = {c: [] for c in cands}
    for fn in cands.values():
        fn(ws[0])
    torch.cuda.synchronize()
    import contextlib
    ctx = contextlib.nullcontext()
    if a.spinner:
        from hwq_probe import SpinnerProc
        ctx = SpinnerProc(20, 4)
    with ctx:
        _rounds(cands, res, ws, it)
    for c, v in res.items():
        t = statistics.median(v)
        print(f"{'[spinner] ' if a.spinner else ''}{c:28s} {t:7.1f} us  {2.0 * m * n * k / t / 1e6:6.0f} TF/s  "
              f"{n * k * 2 / t / 1e6:5.2f} TB/s", flush=True)


def _rounds(cands, res, ws, it):
    for _ in range(5):
        for c, fn in cands.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(6):
                it[0] += 1
                fn(ws[it[0] % 3])
            e1.record()
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) * 1e3 / 6)


if __name__ == "__main__":
    main()
