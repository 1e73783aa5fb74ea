"""Decode LM head (Llama-3-8B: 128,256 x 4,096, M = 256) on each candidate kernel, us per call over
rotating weight copies (each call streams its weight from HBM, as a decode step does).

    python bench/debug/lm_head_bench.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd.ops import gemm


def main():
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
    }
    res = {c: [] for c in cands}
    for fn in cands.values():
        fn(ws[0])
    torch.cuda.synchronize()
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
    for c, v in res.items():
        t = statistics.median(v)
        print(f"{c:28s} {t:7.1f} us  {2.0 * m * n * k / t / 1e6:6.0f} TF/s  {n * k * 2 / t / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
